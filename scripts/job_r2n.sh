#!/bin/bash
# General-geometry Q6 at 1 wave/SIMD (no spills, AGPRs) vs default, and fused4
# 2x8 / 8x2 tiles vs 4x4.
source scripts/gpu_steps.sh
B="python -u bench.py --steps 50 --warmup 5 --extras off --profile-steps 0"
for rep in 1 2; do
  for k in fused2 fused3; do
    step g6_${k}_def_$rep 200 $B --config q6 --perturb 0.1 --kernel $k
    BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_gw1.so step g6_${k}_w1_$rep 200 $B --config q6 --perturb 0.1 --kernel $k
  done
  step q3_44_$rep 200 $B
  BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_t2x8.so step q3_28_$rep 200 $B
  BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_t8x2.so step q3_82_$rep 200 $B
done
python - <<'PY'
import glob, json
for f in sorted(glob.glob('gpurun_out/g6_*.log') + glob.glob('gpurun_out/q3_*.log')):
    for l in open(f):
        if l.startswith('{'):
            d = json.loads(l)
            print(f.split('/')[-1][:-4], round(d['value'], 2), d['config']['kernel'], d['config']['y_norm'])
PY
