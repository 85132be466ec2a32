#!/bin/bash
# fused5 table-row laundering distance: 2 (default) vs 3 / 4 rows in flight.
source scripts/gpu_steps.sh
BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_ld4.so step t_ld4 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py -k "fused5 and (3 or 6)" -m gpu
CFGS="q3 q6 q6f32" VARIANTS="new ld3 ld4" REPS=2 BENCH_EXTRA="--extras off" bash scripts/job_abvar.sh
