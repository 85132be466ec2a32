#!/bin/bash
# r-update pass attribution: kernel time with the fold / r.r dropped (timing only).
# Build the variants first:
#   for v in 1 2 3; do python -m benchmark_dolfinx_amd.ops.build --variant ud$v="-DBDX_UPD_DROP=$v" --only lap_fused4_f64_p3; done
source scripts/gpu_steps.sh
for v in new ud1 ud2 ud3; do
  if [ $v = new ]; then lib=""; else lib=benchmark_dolfinx_amd/ops/libbdx_hip_$v.so; fi
  BDX_HIP_LIB=$lib step ud_$v 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ud_$v -o trace -- python3 bench.py --steps 20 --warmup 2 --config q3
done
