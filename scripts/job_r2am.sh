#!/bin/bash
# fused5 z-pass split (zK written back before zM is formed: 188 -> 170 VGPRs
# in the Q6 FP64 CG instance) and the 3-wave builds it enables.
source scripts/gpu_steps.sh
step t_f5 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py tests/test_gpu_determinism.py -k "fused5" -m gpu
BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_w3e5.so step t_w3e5 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py -k "fused5 and 6 and float64" -m gpu
CFGS="q6" VARIANTS="zs0 new w3e5 w3e7" REPS=2 BENCH_EXTRA="--extras off" bash scripts/job_abvar.sh
CFGS="q6f32" VARIANTS="zs0 new" REPS=2 BENCH_EXTRA="--extras off" bash scripts/job_abvar.sh
