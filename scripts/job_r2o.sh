#!/bin/bash
# fused5 1D tables read from LDS (variant tlds) vs scalar loads (default).
source scripts/gpu_steps.sh
BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_tlds.so step pytest_tlds 300 python -u -m pytest tests/test_gpu_fused.py -q -rf --timeout 240 --timeout-method thread -k "fused5_action and 6-"
CFGS="q6 q6f32" VARIANTS="new tlds" REPS=2 BENCH_EXTRA="--extras off --profile-steps 0" bash scripts/job_abvar.sh
