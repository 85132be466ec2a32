#!/bin/bash
# Validation of the fractional-round segment model: GPU suite, smoke, the
# driver's default bench, and the box / perturbed configs with their chosen S.
source scripts/gpu_steps.sh
step be_pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
step be_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step be_bench_default 600 python -u bench.py
for rep in 1 2; do
  for c in q6 q6f32; do
    step be_${c}_$rep 300 python -u bench.py --config $c --extras off
  done
  for c in q3 q6 q6f32; do
    step be_${c}_pert_$rep 300 python -u bench.py --config $c --perturb 0.1 --extras off
  done
done
