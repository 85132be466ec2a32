#!/bin/bash
# Descriptor laundering in fused3/4/5: correctness (fused GPU suite), then
# interleaved A/B against the un-laundered build (old) on q3 / q6 / q6f32 and
# the general-geometry (perturbed mesh) q3 / q6 paths.
source scripts/gpu_steps.sh
step t_fused 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py tests/test_gpu_runtime.py -m gpu
CFGS="q3 q6 q6f32" VARIANTS="old new" REPS=2 BENCH_EXTRA="--extras off --steps 100" bash scripts/job_abvar.sh
for rep in 1 2; do
  for v in old new; do
    if [ "$v" = new ]; then lib=""; else lib=benchmark_dolfinx_amd/ops/libbdx_hip_$v.so; fi
    BDX_HIP_LIB=$lib step gen_q3_${v}_$rep 300 python -u bench.py --config q3 --perturb 0.1 --steps 30 --warmup 3 --extras off
    BDX_HIP_LIB=$lib step gen_q6_${v}_$rep 300 python -u bench.py --config q6 --perturb 0.1 --steps 30 --warmup 3 --extras off
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
