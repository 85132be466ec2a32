#!/bin/bash
# FP32 fused5 packed-math even-odd products (BDX_F5_PK): correctness (fused5
# suite, all P / precisions) and Q6 FP32 A/B against the scalar build (pk0).
source scripts/gpu_steps.sh
step t_f5 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py tests/test_gpu_determinism.py -k "fused5" -m gpu
CFGS="q6f32" VARIANTS="pk0 new" REPS=3 BENCH_EXTRA="--extras off" bash scripts/job_abvar.sh
