#!/bin/bash
# Full round check on one MI355X: GPU test suite, smoke, headline bench for
# every config, rocprofv3 kernel-trace stats of the default Q3/Q6 paths.
source scripts/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_q3 400 python -u bench.py --config q3 --steps 200 --warmup 10
step bench_q6 400 python -u bench.py --config q6 --steps 200 --warmup 10
step bench_q6f32 400 python -u bench.py --config q6f32 --steps 200 --warmup 10
for c in q3 q6; do
  step trace_$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$c -o trace -- python3 bench.py --steps 20 --warmup 2 --config $c
done
