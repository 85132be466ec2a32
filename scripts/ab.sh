#!/bin/bash
# Interleaved same-box A/B of variant libraries against the production build.
#   [AB_REPS=n] bash scripts/ab.sh "<bench args>" variant1 [variant2 ...]
# (variant = NAME of benchmark_dolfinx_amd/ops/libbdx_hip_NAME.so, or "prod")
source scripts/gpu_steps.sh
args=$1; shift
tag=$(echo "$args" | tr -c 'a-zA-Z0-9' '_' | cut -c1-40)
for rep in $(seq 1 ${AB_REPS:-2}); do
  for v in prod "$@"; do
    if [ "$v" = prod ]; then
      step ab_${tag}_${v}_$rep 300 python -u bench.py $args
    else
      step ab_${tag}_${v}_$rep 300 env BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_$v.so BDX_ALLOW_VARIANT=1 python -u bench.py $args
    fi
    tail -1 gpurun_out/ab_${tag}_${v}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('AB', '$tag', '$v', $rep, round(d['value'],3), round(d['ms_per_step_median'],4))" | tee -a gpurun_out/ab_summary.txt
  done
done
