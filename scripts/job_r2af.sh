#!/bin/bash
# fused3 general geometry (Q3, --perturb 0.1): x-loop unroll 1/2 and 3 waves/SIMD vs the default full unroll at 2 waves.
source scripts/gpu_steps.sh
BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_u1w3.so step t_u1w3 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py -k "fused3 and 3" -m gpu
CFGS="q3" VARIANTS="new u1 u1w3 u2w3" REPS=2 BENCH_EXTRA="--extras off --perturb 0.1 --steps 30 --warmup 3" bash scripts/job_abvar.sh
