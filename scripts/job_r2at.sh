#!/bin/bash
# Q6 FP64 fused5 (y, z) tile in cells: 2x2 (default, 2 workgroups of 4 waves
# per CU) vs 2x4 (1 workgroup of 8 waves), 1x2 (4 of 2), 1x4 (2 of 4).
source scripts/gpu_steps.sh
BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_t12.so step t_t12 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py -k "fused5 and 6 and float64" -m gpu
CFGS="q6" VARIANTS="new t24 t12 t14" REPS=2 BENCH_EXTRA="--extras off" bash scripts/job_abvar.sh
