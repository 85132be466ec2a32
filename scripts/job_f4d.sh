#!/bin/bash
source scripts/gpu_steps.sh
step pytest_f4 600 python -u -m pytest tests/test_gpu_fused.py -q --timeout 120 --timeout-method thread -k "fused4 or sheared"
step bench_q3_f4 400 python -u bench.py --config q3 --steps 200 --warmup 10 --kernel fused4
step bench_q3_f4_rand 400 python -u bench.py --config q3 --steps 200 --warmup 10 --kernel fused4 --kappa random
step trace_q3_f4 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_q3_f4 -o trace -- python3 bench.py --steps 20 --warmup 2 --config q3 --kernel fused4
