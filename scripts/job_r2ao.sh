#!/bin/bash
# fused3 general geometry after moving the coefficient / vertex prefetch
# ahead of the vector batch: staging-first (sf3) and 2-wave (w2) variants.
source scripts/gpu_steps.sh
step t_f3 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py tests/test_gpu_determinism.py -k "fused3" -m gpu
BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_sf3.so step t_sf3 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py -k "fused3 and (3 or 6)" -m gpu
for rep in 1 2; do
  for v in new sf3 w2 sf3w2; do
    if [ "$v" = new ]; then lib=""; else lib=benchmark_dolfinx_amd/ops/libbdx_hip_$v.so; fi
    for cfg in q3 q6; do
      BDX_HIP_LIB=$lib step gen_${cfg}_${v}_$rep 300 python -u bench.py --config $cfg --perturb 0.1 --steps 30 --warmup 3 --extras off
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
            res[f.split('/')[-1][:-4].rsplit('_', 1)[0]].append(round(d['value'], 2))
for k, v in sorted(res.items()):
    print(k, v)
PY
