#!/bin/bash
# fused4 element-vector pitches (4, 17, 72) vs (5, 21, 85): numerics + same-box A/B
source scripts/gpu_steps.sh
step pytest_f4p 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_distributed_emulated.py -q -x --timeout 120 --timeout-method thread -k "fused4 or q3 or 3-"
CFGS="q3" VARIANTS="p0 new" REPS=3 bash scripts/job_abvar.sh
