#!/bin/bash
# fused5 descriptor laundering + single table base: correctness, then
# interleaved A/B (old = no laundering, w3 = 3 waves/SIMD, eo7 = FP64 even-odd on all passes).
source scripts/gpu_steps.sh
step t_f5 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py -k "fused5" -m gpu
CFGS="q6 q6f32" VARIANTS="old new w3 eo7" REPS=2 BENCH_EXTRA="--extras off" bash scripts/job_abvar.sh
