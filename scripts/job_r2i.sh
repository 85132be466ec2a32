#!/bin/bash
# (1) full GPU suite on the 3-wave fused4 default; (2) fused4 phase-drop
# attribution (timing only, wrong numerics: BDX_ALLOW_DROP); (3) general-
# geometry kernels at 2 waves/SIMD (variant gw2) vs the default 3 (Q3) / 2 (Q6).
source scripts/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread
B="python -u bench.py --steps 50 --warmup 5 --extras off --profile-steps 0"
step f4_base 200 $B
for d in 1 2 4 8; do
  BDX_ALLOW_DROP=1 BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_f4d$d.so step f4_drop$d 200 $B
done
step f4_base2 200 $B
for k in fused2 fused3; do
  step gen_q3_${k}_w3 200 $B --perturb 0.1 --kernel $k
  BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_gw2.so step gen_q3_${k}_w2 200 $B --perturb 0.1 --kernel $k
  step gen_q6_${k}_def 200 $B --config q6 --perturb 0.1 --kernel $k
  BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_gw2.so step gen_q6_${k}_w2 200 $B --config q6 --perturb 0.1 --kernel $k
done
python - <<'PY'
import glob, json
for f in sorted(glob.glob('gpurun_out/f4_*.log') + glob.glob('gpurun_out/gen_*.log')):
    for l in open(f):
        if l.startswith('{'):
            d = json.loads(l)
            print(f.split('/')[-1][:-4], round(d['value'], 2), round(d['ms_per_step'], 3), d['config']['kernel'])
PY
