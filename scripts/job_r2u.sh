#!/bin/bash
# GPU suite on the tiled build; kernel-trace profiles of Q3 / Q6 (tiled).
source scripts/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread
step trace_q3 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_q3t -o trace -- python3 bench.py --steps 20 --warmup 2 --profile-steps 0 --extras off
step trace_q6 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_q6t -o trace -- python3 bench.py --config q6 --steps 20 --warmup 2 --profile-steps 0 --extras off
