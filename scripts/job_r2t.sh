#!/bin/bash
# Tiled vector storage in the native CG runtime: GPU suite (incl. the
# tiled-vs-lattice tests), then an interleaved A/B of the headline configs.
source scripts/gpu_steps.sh
step pytest_tiled 600 python -u -m pytest tests/test_gpu_runtime.py -q -rf --timeout 240 --timeout-method thread -k "tiled"
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread
B="python -u bench.py --steps 50 --warmup 5 --extras off --profile-steps 0"
for rep in 1 2; do
  for cfg in q3 q6 q6f32; do
    BDX_TILED=0 step ab_${cfg}_lat_$rep 200 $B --config $cfg
    BDX_TILED=1 step ab_${cfg}_til_$rep 200 $B --config $cfg
  done
done
python - <<'PY'
import glob, json
for f in sorted(glob.glob('gpurun_out/ab_*.log')):
    for l in open(f):
        if l.startswith('{'):
            d = json.loads(l)
            print(f.split('/')[-1][:-4], round(d['value'], 2), round(d['ms_per_step'], 3), d['config']['y_norm'], d['config']['runtime'])
PY
