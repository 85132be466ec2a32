#!/bin/bash
# fused4 (MFMA Kronecker core) validation + A/B against fused3.
source scripts/gpu_steps.sh
step pytest_f4 600 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread -k "fused4 or 4-True or version4 or -4-"
step bench_q3_f4 300 python -u bench.py --steps 100 --warmup 5 --kernel fused4
step bench_q3_f3 300 python -u bench.py --steps 100 --warmup 5 --kernel fused3
step prof_q3_f4 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f4 -o f4 -- python3 bench.py --steps 20 --warmup 2 --kernel fused4
