#!/bin/bash
# Flat r-update grid cap (partials count) A/B: 65536 (default) vs 16384 vs 8192 vs the row kernel.
source scripts/gpu_steps.sh
CFGS="q3 q6" VARIANTS="row new g16384 g8192" REPS=2 bash scripts/job_abvar.sh
for v in g8192 g16384; do
  BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_$v.so step ug_prof_$v 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ug_$v -o trace -- python3 bench.py --steps 20 --warmup 2 --config q3
done
