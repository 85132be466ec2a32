#!/bin/bash
# r-update pass attribution: kernel time with the fold / r.r dropped (timing only).
source scripts/gpu_steps.sh
for v in new ud1 ud2 ud3; do
  if [ $v = new ]; then lib=""; else lib=benchmark_dolfinx_amd/ops/libbdx_hip_$v.so; fi
  BDX_HIP_LIB=$lib step ud_$v 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ud_$v -o trace -- python3 bench.py --steps 20 --warmup 2 --config q3
done
