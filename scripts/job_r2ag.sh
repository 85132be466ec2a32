#!/bin/bash
# fused3 general geometry with the rolled x loop and 3 waves/SIMD (new
# defaults) vs the previous build (old): correctness, then A/B on perturbed
# meshes at Q3 / Q6 FP64 and Q3 / Q6 FP32.
source scripts/gpu_steps.sh
step t_fused3 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py tests/test_gpu_determinism.py -k "fused3 or fused2" -m gpu
for rep in 1 2; do
  for v in old new; do
    if [ "$v" = new ]; then lib=""; else lib=benchmark_dolfinx_amd/ops/libbdx_hip_$v.so; fi
    for cfg in q3 q6 q6f32; do
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
