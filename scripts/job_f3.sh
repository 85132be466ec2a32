#!/bin/bash
source scripts/gpu_steps.sh
step pytest_fused 900 python -m pytest tests/test_gpu_fused.py -x -q
for c in q3 q6; do
  for k in fused2 fused3; do
    step bench_${c}_$k 300 python -u bench.py --steps 20 --warmup 3 --config $c --kernel $k
  done
done
step bench_q3_f3gen 300 python -u bench.py --steps 20 --warmup 3 --config q3 --kernel fused3 --geometry otf-general
step bench_q6_f3gen 300 python -u bench.py --steps 20 --warmup 3 --config q6 --kernel fused3 --geometry otf-general
step bench_q6f32_f3 300 python -u bench.py --steps 20 --warmup 3 --config q6f32 --kernel fused3
grep -h '^{' gpurun_out/bench_*.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['config']['model'][:3], d['dtype'], d['config']['kernel'], d['config']['geometry'], round(d['value'], 3), round(d['ms_per_step'], 3), d['config']['y_norm'])
" || true
