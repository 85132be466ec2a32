#!/bin/bash
# Stage attribution of fused3 on general (trilinear) meshes, Q6 and Q3
# (timing only, wrong numerics: BDX_ALLOW_DROP=1), plus the determinism tests.
source scripts/gpu_steps.sh
step pytest_det 300 python -u -m pytest tests/test_gpu_determinism.py -q -rf --timeout 240 --timeout-method thread
for cfg in q6 q3; do
  B="python -u bench.py --config $cfg --steps 30 --warmup 3 --extras off --profile-steps 0 --perturb 0.1 --kernel fused3"
  step a_${cfg}_base 200 $B
  for v in x3fz x3fy x3xf x3by x3bz x3sy x3st x3out; do
    BDX_ALLOW_DROP=1 BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_$v.so step a_${cfg}_$v 200 $B
  done
done
python - <<'PY'
import glob, json
for f in sorted(glob.glob('gpurun_out/a_*.log')):
    for l in open(f):
        if l.startswith('{'):
            d = json.loads(l)
            print(f.split('/')[-1][:-4], round(d['ms_per_step'], 3), d['config']['build_flags']['drops'])
PY
