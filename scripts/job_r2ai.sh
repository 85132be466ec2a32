#!/bin/bash
# fused3 on the runtime's tiled storage: runtime + fused3 tests, then general
# geometry A/B, tiled (default) vs lattice layout (BDX_TILED=0), same library.
source scripts/gpu_steps.sh
step t_rt 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_runtime.py -m gpu
for rep in 1 2; do
  for t in 0 1; do
    for cfg in q3 q6 q6f32; do
      BDX_TILED=$t step gen_${cfg}_t${t}_$rep 300 python -u bench.py --config $cfg --perturb 0.1 --steps 30 --warmup 3 --extras off
    done
  done
done
python - <<'PY'
import glob, json, collections
res = collections.defaultdict(list)
for f in sorted(glob.glob('gpurun_out/gen_*.log')):
    for l in open(f):
        if l.startswith('{'):
            d = json.loads(l)
            res[f.split('/')[-1][:-4].rsplit('_', 1)[0]].append((round(d['value'], 2), d['config']['runtime']))
for k, v in sorted(res.items()):
    print(k, v)
PY
