#!/bin/bash
# fused4/fused5 store/prefetch wait restructuring: numerics, then same-box A/B vs HEAD.
source scripts/gpu_steps.sh
step pytest_f45 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_distributed_emulated.py -q -x --timeout 120 --timeout-method thread
bash scripts/job_abhead.sh
