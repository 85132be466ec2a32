#!/bin/bash
# Line-aligned tile shapes: fused4 1x16 / 2x16 cells (48-node = 384-byte owned
# z rows: whole 128-byte lines per tile) and fused5 Q6 1x8 (FP64 rows 384 B)
# vs the default 4x4 / 2x2 tiles; correctness of the variants first.
source scripts/gpu_steps.sh
for v in t1x16 t2x16; do
  BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_$v.so step pytest_$v 300 python -u -m pytest tests/test_gpu_fused.py -q -rf --timeout 240 --timeout-method thread -k "fused4 and not segments"
done
BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_t1x8.so step pytest_t1x8 300 python -u -m pytest tests/test_gpu_fused.py -q -rf --timeout 240 --timeout-method thread -k "fused5 and not segments"
CFGS="q3" VARIANTS="new t1x16 t2x16" REPS=2 BENCH_EXTRA="--extras off --profile-steps 0" bash scripts/job_abvar.sh
CFGS="q6 q6f32" VARIANTS="new t1x8" REPS=2 BENCH_EXTRA="--extras off --profile-steps 0" bash scripts/job_abvar.sh
