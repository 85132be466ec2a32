#!/bin/bash
# fused5 FP32 2-array instances at 3 waves/SIMD: numerics + same-box A/B vs HEAD
source scripts/gpu_steps.sh
step pytest_w3 600 python -u -m pytest tests/test_gpu_fused.py -q -x --timeout 120 --timeout-method thread
CFGS="q6f32" VARIANTS="head new" REPS=3 bash scripts/job_abvar.sh
