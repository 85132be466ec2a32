#!/bin/bash
# Round-3 first GPU call: GPU suite, smoke, default bench (Q3 headline + Q6
# companions), then the per-config base numbers.
source scripts/gpu_steps.sh
step r3_pytest_gpu 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
step r3_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step r3_bench_default 600 python -u bench.py
step r3_base 900 bash scripts/r3_base.sh
