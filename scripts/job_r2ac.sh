#!/bin/bash
# Q3: fused4 (MFMA) vs fused5 (nodal Kronecker, laundered descriptors), interleaved.
source scripts/gpu_steps.sh
for rep in 1 2; do
  step q3f4_$rep 200 python -u bench.py --config q3 --steps 100 --warmup 5 --extras off --kernel fused4
  step q3f5_$rep 200 python -u bench.py --config q3 --steps 100 --warmup 5 --extras off --kernel fused5
done
python - <<'PY'
import glob, json
for f in sorted(glob.glob('gpurun_out/q3f*.log')):
    for l in open(f):
        if l.startswith('{'):
            d = json.loads(l); print(f.split('/')[-1][:-4], round(d['value'], 2), d['config']['phases_ms'])
PY
