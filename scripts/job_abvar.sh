#!/bin/bash
# Same-box interleaved A/B over library variants: VARIANTS="head g x" (libbdx_hip_<v>.so; "new" = libbdx_hip.so)
source scripts/gpu_steps.sh
CFGS=${CFGS:-q6 q6f32}
VARIANTS=${VARIANTS:-head new}
REPS=${REPS:-2}
for cfg in $CFGS; do
  for rep in $(seq $REPS); do
    for v in $VARIANTS; do
      if [ "$v" = new ]; then lib=""; else lib=benchmark_dolfinx_amd/ops/libbdx_hip_$v.so; fi
      BDX_HIP_LIB=$lib step abv_${cfg}_${v}_$rep 300 python -u bench.py --config $cfg --steps 100 --warmup 5 $BENCH_EXTRA
    done
  done
done
python - <<'PY'
import glob, json, collections
res = collections.defaultdict(list)
for f in sorted(glob.glob('gpurun_out/abv_*.log')):
    for l in open(f):
        if l.startswith('{'):
            d = json.loads(l)
            key = f.split('/')[-1][4:-4].rsplit('_', 1)[0]
            res[key].append(round(d['value'], 2))
for k, v in sorted(res.items()):
    print(k, v, 'mean', round(sum(v) / len(v), 2))
PY
