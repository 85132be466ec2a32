#!/bin/bash
# Round re-entry validation: GPU tests, smoke, the three bench configs.
source scripts/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_q3 300 python -u bench.py --steps 200 --warmup 10
step bench_q6 300 python -u bench.py --config q6 --steps 100 --warmup 10
step bench_q6f32 300 python -u bench.py --config q6f32 --steps 100 --warmup 10
step bench_q3_kr 300 python -u bench.py --steps 200 --warmup 10 --kappa random
