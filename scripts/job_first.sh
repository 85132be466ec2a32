#!/bin/bash
# First end-to-end GPU session: build, GPU tests, smoke, Q3/Q6 bench, kernel profile.
source scripts/gpu_steps.sh
step build 600 python -c "import __graft_entry__ as g; g.build()"
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -m pytest tests -m gpu -x -q
step bench_q3 600 python -u bench.py --steps 20 --warmup 3 --config q3
step bench_q6 600 python -u bench.py --steps 20 --warmup 3 --config q6
step prof_q3 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_q3 -o trace -- python3 bench.py --steps 10 --warmup 2 --config q3
