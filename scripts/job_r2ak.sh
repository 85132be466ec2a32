#!/bin/bash
# fused5 Q6 FP64: gather sources recomputed per layer (orc) and 3 waves/SIMD
# (orcw3e5: spill-free with even-odd on x/y; orcw3e7: 10-dword spill).
source scripts/gpu_steps.sh
BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_orcw3e5.so step t_w3 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py -k "fused5 and 6 and float64" -m gpu
CFGS="q6" VARIANTS="new orc orcw3e5 orcw3e7" REPS=2 BENCH_EXTRA="--extras off" bash scripts/job_abvar.sh
