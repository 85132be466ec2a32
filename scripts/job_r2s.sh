#!/bin/bash
# fused4 attribution, second pass: barriers dropped (16), loads + gather
# dropped together (6), everything but the staging dropped (7).
source scripts/gpu_steps.sh
B="python -u bench.py --steps 50 --warmup 5 --extras off --profile-steps 0"
step f4_base 200 $B
for d in 16 6 7; do
  BDX_ALLOW_DROP=1 BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_f4d$d.so step f4_drop$d 200 $B
done
step f4_base2 200 $B
step prof_q3 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_q3 -o trace -- python3 bench.py --steps 20 --warmup 2 --profile-steps 0 --extras off
python - <<'PY'
import glob, json
for f in sorted(glob.glob('gpurun_out/f4_*.log')):
    for l in open(f):
        if l.startswith('{'):
            d = json.loads(l)
            print(f.split('/')[-1][:-4], round(d['value'], 2), round(d['ms_per_step'], 3))
PY
