#!/bin/bash
source scripts/gpu_steps.sh
step pytest_gpu 1200 python -m pytest tests -m gpu -x -q
for c in q3 q6; do
  step bench_${c}_const 300 python -u bench.py --steps 30 --warmup 3 --config $c
  step bench_${c}_rand 300 python -u bench.py --steps 30 --warmup 3 --config $c --kappa random
done
grep -h '^{' gpurun_out/bench_*.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['config']['model'][:3], d['dtype'], d['config']['kernel'], d['config']['kappa'], round(d['value'], 3), round(d['ms_per_step'], 3), d['config']['y_norm'])
" || true
