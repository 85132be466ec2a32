#!/bin/bash
# A/B of kernel variants (libbdx_hip_<v>.so) on one config and kernel:
#   VARIANTS="base d1 ..." CFG=q3 KERNEL=fused4 bash scripts/job_ab.sh
source scripts/gpu_steps.sh
for v in ${VARIANTS:-base}; do
  lib=""
  [ "$v" != base ] && lib=$PWD/benchmark_dolfinx_amd/ops/libbdx_hip_$v.so
  step ab_${CFG:-q3}_$v 120 env BDX_HIP_LIB=$lib python -u bench.py --steps ${STEPS:-30} --warmup 3 --config ${CFG:-q3} --kernel ${KERNEL:-auto}
done
grep -h '^{' gpurun_out/ab_*.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['config']['model'][:3], d['config']['kernel'], d['config'].get('hiplib', ''), round(d['value'], 3), round(d['ms_per_step'], 3))
" || true
