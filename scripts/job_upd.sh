#!/bin/bash
source scripts/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
CFGS="q3 q6" VARIANTS="head new" bash scripts/job_abvar.sh
step prof_upd_q6 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_upd_q6 -o t -- python3 bench.py --steps 20 --warmup 2 --config q6
step prof_upd_q3 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_upd_q3 -o t -- python3 bench.py --steps 20 --warmup 2 --config q3
