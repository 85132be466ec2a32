#!/bin/bash
# fused5 staging before the gather with one explicit vmcnt(0) (sf) vs the
# default order (gather, then staging: each slot's wait drains the stores).
source scripts/gpu_steps.sh
BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_sf.so step t_sf 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py -k "fused5 and (3 or 6)" -m gpu
CFGS="q3 q6 q6f32" VARIANTS="new sf" REPS=2 BENCH_EXTRA="--extras off" bash scripts/job_abvar.sh
