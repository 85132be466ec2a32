#!/bin/bash
# fused5 even-odd rows from the interleaved (E, O) table block (one scalar
# load per row pair) vs separate E / O rows (eor0); fused5 tests on the default.
source scripts/gpu_steps.sh
step t_f5 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py tests/test_gpu_determinism.py -k "fused5" -m gpu
CFGS="q3 q6 q6f32" VARIANTS="eor0 new" REPS=2 BENCH_EXTRA="--extras off" bash scripts/job_abvar.sh
