#!/bin/bash
# kc prefetch + LDS-only wave fences: fused4/fused5 numerics and A/B.
source scripts/gpu_steps.sh
step pytest_f45 600 python -u -m pytest tests/test_gpu_fused.py -q -x --timeout 120 --timeout-method thread -k "fused4 or fused5 or 5-True or -5-"
step kc_q3 300 python -u bench.py --config q3 --steps 100 --warmup 5
step kc_q6 300 python -u bench.py --config q6 --steps 100 --warmup 5
step kc_q6f32 300 python -u bench.py --config q6f32 --steps 100 --warmup 5
step kc_q3r 300 python -u bench.py --config q3 --steps 100 --warmup 5 --kappa random
step prof_kc_q6 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kc_q6 -o t -- python3 bench.py --steps 20 --warmup 2 --config q6
grep -h '^{' gpurun_out/kc_*.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); c = d['config']; print(c['model'][:3], d['dtype'], c['kernel'], c['kappa'], round(d['value'], 3), round(d['ms_per_step'], 3))
"
