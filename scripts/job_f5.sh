#!/bin/bash
# fused5 (nodal Kronecker core): numerics + A/B against fused3/fused4.
source scripts/gpu_steps.sh
step pytest_f5 600 python -u -m pytest tests/test_gpu_fused.py -q --timeout 120 --timeout-method thread -k "fused5 or 5-True or -5-"
for k in fused3 fused5; do
  step ab_q6_$k 300 python -u bench.py --config q6 --steps 50 --warmup 5 --kernel $k
  step ab_q6f32_$k 300 python -u bench.py --config q6f32 --steps 50 --warmup 5 --kernel $k
done
for k in fused4 fused5; do
  step ab_q3_$k 300 python -u bench.py --config q3 --steps 50 --warmup 5 --kernel $k
done
grep -h '^{' gpurun_out/ab_*.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); c = d['config']; print(c['model'][:3], d['dtype'], c['kernel'], round(d['value'], 3), round(d['ms_per_step'], 3), repr(c['y_norm']))
"
