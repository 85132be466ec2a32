#!/bin/bash
# Same-box A/B of the working tree (libbdx_hip.so) against a reference build
# (libbdx_hip_head.so from scripts/build_ref_variant.sh), interleaved.
source scripts/gpu_steps.sh
CFGS=${CFGS:-q3 q6 q6f32}
for cfg in $CFGS; do
  for rep in 1 2; do
    BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_head.so step abh_${cfg}_head_$rep 300 python -u bench.py --config $cfg --steps 100 --warmup 5 $BENCH_EXTRA
    step abh_${cfg}_new_$rep 300 python -u bench.py --config $cfg --steps 100 --warmup 5 $BENCH_EXTRA
  done
done
for f in gpurun_out/abh_*.log; do
  python -c "
import sys, json
for l in open('$f'):
    if l.startswith('{'):
        d = json.loads(l); c = d['config']; print('$f'.split('/')[-1][:-4], c['kernel'], round(d['value'], 3), round(d['ms_per_step'], 3))
"
done
