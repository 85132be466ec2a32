#!/bin/bash
# Round-2 first GPU pass: full GPU suite, then the headline benches.
source scripts/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread
step bench_q3 300 python bench.py --steps 20 --warmup 5
step bench_q6 300 python bench.py --config q6 --steps 20 --warmup 5
