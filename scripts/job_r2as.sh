#!/bin/bash
# Tiled r update: z index stepped per element (new) vs recomputed per element (upd0).
source scripts/gpu_steps.sh
step t_rt 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_runtime.py tests/test_gpu_determinism.py -m gpu
CFGS="q6f32 q6 q3" VARIANTS="upd0 new" REPS=2 BENCH_EXTRA="--extras off" bash scripts/job_abvar.sh
for v in upd0 new; do
  if [ "$v" = new ]; then lib=""; else lib=benchmark_dolfinx_amd/ops/libbdx_hip_$v.so; fi
  python - "$v" <<'PY'
import glob, json, sys
for f in sorted(glob.glob(f'gpurun_out/abv_*_{sys.argv[1]}_1.log')):
    for l in open(f):
        if l.startswith('{'):
            d = json.loads(l); print(f.split('/')[-1], 'update_rr ms', round(d['config']['phases_ms']['update_rr'], 3))
PY
done
