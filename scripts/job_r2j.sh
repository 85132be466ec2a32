#!/bin/bash
# Non-temporal stream loads/stores (default build) vs default cache policy
# (variant nt0): GPU suite, then interleaved A/B on the three headline configs.
source scripts/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread
CFGS="q3 q6 q6f32" VARIANTS="nt0 new" REPS=2 BENCH_EXTRA="--extras off --profile-steps 0" bash scripts/job_abvar.sh
