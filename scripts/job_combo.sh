#!/bin/bash
# pytest (fused + emulated multi-rank) then kernel-variant A/B
source scripts/gpu_steps.sh
step pytest_fused 900 python -m pytest tests/test_gpu_fused.py tests/test_gpu_distributed_emulated.py -x -q
bash scripts/job_variants.sh
