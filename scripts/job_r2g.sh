#!/bin/bash
# Full-size CG iterate pin (production vs stored-G v1) and bench.py with the
# random-kappa / general-geometry variants.
source scripts/gpu_steps.sh
step pytest_fullsize 600 python -u -m pytest tests/test_gpu_fullsize_cg.py -v -s --timeout 300 --timeout-method thread
step bench_q3 300 python bench.py --steps 50 --warmup 5
step bench_q6 300 python bench.py --config q6 --steps 50 --warmup 5
step trace_q3 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_q3 -o trace -- python3 bench.py --steps 20 --warmup 2 --profile-steps 0 --extras off
