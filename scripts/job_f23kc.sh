#!/bin/bash
# fused2/fused3 kc prefetch: numerics + same-box A/B (fused3 and general-geometry fused2 paths)
source scripts/gpu_steps.sh
step pytest_f23 600 python -u -m pytest tests/test_gpu_fused.py -q -x --timeout 120 --timeout-method thread
CFGS="q3 q6" VARIANTS="head new" BENCH_EXTRA="--kernel fused3" bash scripts/job_abvar.sh
mkdir -p gpurun_out/g && mv gpurun_out/abv_* gpurun_out/g/
CFGS="q3" VARIANTS="head new" BENCH_EXTRA="--kernel fused2 --geometry otf-general" bash scripts/job_abvar.sh
