#!/bin/bash
source scripts/gpu_steps.sh
step pytest_f4 600 python -u -m pytest tests/test_gpu_fused.py -q --timeout 120 --timeout-method thread -k "fused4 or 4-True or -4- or sheared"
VARIANTS="base noskip" KERNEL=fused4 bash scripts/job_ab.sh
