#!/bin/bash
# RCCL transport self-test on the box's GPU, then fused4 tile-shape A/B (4x4 vs 4x8 vs 8x4 cells).
source scripts/gpu_steps.sh
step pytest_rccl 300 python -u -m pytest tests/test_gpu_rccl.py -v --timeout 120 --timeout-method thread
CFGS="q3" VARIANTS="new tz8 ty8" REPS=2 bash scripts/job_abvar.sh
