#!/bin/bash
# Q3 fused5 (y, z) tile: 4x4 (default) vs 4x8 vs 8x4 cells per workgroup, plus a fused5 correctness pass per tile.
source scripts/gpu_steps.sh
BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_t48.so step t_t48 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py -k "fused5 and 3" -m gpu
BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_t84.so step t_t84 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py -k "fused5 and 3" -m gpu
CFGS="q3" VARIANTS="new t48 t84" REPS=2 BENCH_EXTRA="--extras off" bash scripts/job_abvar.sh
