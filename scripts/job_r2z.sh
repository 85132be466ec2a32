#!/bin/bash
# fused4 on the tiled runtime: prefetch depth 1 vs 2, 3 vs 2 waves per SIMD.
source scripts/gpu_steps.sh
B="python -u bench.py --steps 100 --warmup 5 --extras off --profile-steps 0"
for rep in 1 2; do
  step d1w3_$rep 200 $B
  BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_w2.so step d1w2_$rep 200 $B
  BDX_F4_DEPTH=2 BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_w2.so step d2w2_$rep 200 $B
done
python - <<'PY'
import glob, json
for f in sorted(glob.glob('gpurun_out/d*w*.log')):
    for l in open(f):
        if l.startswith('{'):
            d = json.loads(l)
            print(f.split('/')[-1][:-4], round(d['value'], 2))
PY
