#!/bin/bash
# Flat non-persistent r-update (BDX_UPD_FLAT=1) vs the row kernel: GPU suite, A/B, kernel times.
source scripts/gpu_steps.sh
step pytest_uf2 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
CFGS="q3 q6 q6f32" VARIANTS="row new" REPS=2 bash scripts/job_abvar.sh
for v in new row; do
  if [ $v = new ]; then lib=""; else lib=benchmark_dolfinx_amd/ops/libbdx_hip_$v.so; fi
  BDX_HIP_LIB=$lib step uf2_prof_$v 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/uf2_$v -o trace -- python3 bench.py --steps 20 --warmup 2 --config q3
done
