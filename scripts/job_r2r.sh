#!/bin/bash
# fused3 general instances with per-layer recomputed output descriptors
# (default) vs resident descriptors (variant orc0): tests, then A/B.
source scripts/gpu_steps.sh
step pytest_f3 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_kernels.py tests/test_gpu_runtime.py -q -rf --timeout 240 --timeout-method thread -k "fused3 or version3 or -3- or general or pert"
for rep in 1 2; do
  for cfg in q6 q3; do
    B="python -u bench.py --config $cfg --steps 30 --warmup 3 --extras off --profile-steps 0 --perturb 0.1 --kernel fused3"
    step g_${cfg}_new_$rep 200 $B
    BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_orc0.so step g_${cfg}_old_$rep 200 $B
  done
done
python - <<'PY'
import glob, json
for f in sorted(glob.glob('gpurun_out/g_*.log')):
    for l in open(f):
        if l.startswith('{'):
            d = json.loads(l)
            print(f.split('/')[-1][:-4], round(d['value'], 2), d['config']['y_norm'])
PY
