#!/bin/bash
# dofmap (unstructured data model) operator: GPU tests, v1 regression after
# the shared-core refactor, and full-size benches of the indirection cost.
source scripts/gpu_steps.sh
step pytest_dofmap 600 python -u -m pytest tests/test_gpu_dofmap.py tests/test_gpu_kernels.py -q -rf --timeout 240 --timeout-method thread
B="python -u bench.py --steps 20 --warmup 3 --extras off --profile-steps 0"
step q3_dofmap_otf 300 $B --kernel dofmap
step q3_dofmap_stored 300 $B --kernel dofmap --geometry stored
step q3_v1_stored 300 $B --kernel v1 --geometry stored
step q6_dofmap_otf 300 $B --config q6 --kernel dofmap
step q3_dofmap_gen 300 $B --kernel dofmap --perturb 0.1
python - <<'PY'
import glob, json
for f in sorted(glob.glob('gpurun_out/q*.log')):
    for l in open(f):
        if l.startswith('{'):
            d = json.loads(l)
            c = d['config']
            print(f.split('/')[-1][:-4], round(d['value'], 2), round(d['ms_per_step'], 3), c['kernel'], c['geometry'], c['setup_s'])
PY
