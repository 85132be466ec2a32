#!/bin/bash
# A/B the kernel variants built with `build.py --variant NAME=FLAGS`:
#   VARIANTS="base rcp ..." CONFIGS="q3 q6" bash scripts/job_variants.sh
source scripts/gpu_steps.sh
for v in ${VARIANTS:-base}; do
  lib=""
  [ "$v" != base ] && lib=$PWD/benchmark_dolfinx_amd/ops/libbdx_hip_$v.so
  for c in ${CONFIGS:-q3}; do
    step bench_${c}_$v 300 env BDX_HIP_LIB=$lib python -u bench.py --steps ${STEPS:-20} --warmup 3 --config $c
  done
done
for v in ${TESTVARIANTS:-}; do
  step pytest_$v 600 env BDX_HIP_LIB=$PWD/benchmark_dolfinx_amd/ops/libbdx_hip_$v.so python -m pytest tests/test_gpu_fused.py -x -q
done
grep -h '^{' gpurun_out/bench_*.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['config']['model'][:3], d['config'].get('hiplib', ''), round(d['value'], 3), round(d['ms_per_step'], 3))
" || true
