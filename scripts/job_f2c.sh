#!/bin/bash
source scripts/gpu_steps.sh
step pytest_gpu 900 python -m pytest tests -m gpu -x -q
for c in q3 q6; do
  step bench_${c}_f2 300 python -u bench.py --steps 20 --warmup 3 --config $c
done
step bench_q3_f2gen 300 python -u bench.py --steps 20 --warmup 3 --config q3 --geometry otf-general
step prof_f2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_f2c -o trace -- python3 bench.py --steps 10 --warmup 2 --config q3
grep -h '^{' gpurun_out/bench_*.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['config']['model'][:3], d['config']['kernel'], d['config']['geometry'], round(d['value'], 3), round(d['ms_per_step'], 3), d['config']['y_norm'])
" || true
