#!/bin/bash
# Flat, 4-vector-per-thread r-update pass: GPU suite + same-box A/B vs HEAD.
source scripts/gpu_steps.sh
step pytest_updflat 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
CFGS="q3 q6" VARIANTS="head new" REPS=2 bash scripts/job_abvar.sh
step prof_updflat 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_updflat -o trace -- python3 bench.py --steps 20 --warmup 2 --config q3
