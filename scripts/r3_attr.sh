#!/bin/bash
# Round 3: fused5 phase attribution (timing-only drop builds, wrong numerics):
# d1 = no x/z/y passes, d2 = no gather stores, d4 = no next-layer loads.
source scripts/gpu_steps.sh
for cfg in q6 q3 q6f32; do
  for v in prod d1 d2 d4 d6; do
    if [ $v = prod ]; then
      step at_${cfg}_$v 200 python -u bench.py --config $cfg --steps 50 --warmup 5 --companions off --extras off --profile-steps 5
    else
      step at_${cfg}_$v 200 env BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_$v.so BDX_ALLOW_VARIANT=1 python -u bench.py --config $cfg --steps 50 --warmup 5 --companions off --extras off --profile-steps 5
    fi
    tail -1 gpurun_out/at_${cfg}_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['config']['phases_ms']; print('ATTR', '$cfg', '$v', round(d['value'],2), round(p['op_interior'],3), round(p['update_rr'],3), round(p['iteration'],3))" | tee -a gpurun_out/attr_summary.txt
  done
done
