#!/bin/bash
source scripts/gpu_steps.sh
step pytest_fused 900 python -m pytest tests/test_gpu_fused.py tests/test_gpu_distributed_emulated.py -x -q
step bench_q3 300 python -u bench.py --steps 50 --warmup 5 --config q3
step bench_q6 300 python -u bench.py --steps 50 --warmup 5 --config q6
step bench_q3_nograph 300 env BDX_GRAPH=0 python -u bench.py --steps 50 --warmup 5 --config q3
grep -h '^{' gpurun_out/bench_*.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['config']['model'][:3], d['dtype'], d['config']['kernel'], d['config']['runtime'], round(d['value'], 3), round(d['ms_per_step'], 3), d['config']['y_norm'])
" || true
