#!/bin/bash
# Round 3: fused3 phase attribution (timing-only builds, wrong numerics):
# e1 = no front z/y contractions, e2 = no x-column loop (gradient, geometry,
# F, transposed x), e4 = no back y/z contractions, e8 = no loads / gather stores.
source scripts/gpu_steps.sh
for cfg in "q3p:--config q3 --perturb 0.1" "q6p:--config q6 --perturb 0.1" "q3g:--config q3 --perturb 0.1 --geometry otf-general"; do
  name=${cfg%%:*}; args=${cfg#*:}
  for v in prod e1 e2 e4 e8; do
    if [ $v = prod ]; then
      step at3_${name}_$v 200 python -u bench.py $args --steps 30 --warmup 3 --companions off --extras off --profile-steps 3
    else
      step at3_${name}_$v 200 env BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_$v.so BDX_ALLOW_VARIANT=1 python -u bench.py $args --steps 30 --warmup 3 --companions off --extras off --profile-steps 3
    fi
    tail -1 gpurun_out/at3_${name}_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['config']['phases_ms']; print('ATTR3', '$name', '$v', round(d['value'],2), round(p['op_interior'],3), round(p['update_rr'],3), round(p['iteration'],3), d['config']['geometry'])" | tee -a gpurun_out/attr3_summary.txt
  done
done
