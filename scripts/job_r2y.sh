#!/bin/bash
# fused5 even-odd matvecs (default) vs plain (variant eo0): fused5 tests, A/B.
source scripts/gpu_steps.sh
step pytest_f5 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_runtime.py tests/test_gpu_determinism.py -q -rf --timeout 240 --timeout-method thread -k "fused5 or version5 or -5- or golden or tiled or bitwise"
CFGS="q6 q6f32" VARIANTS="eo0 new" REPS=2 BENCH_EXTRA="--extras off --profile-steps 0" bash scripts/job_abvar.sh
