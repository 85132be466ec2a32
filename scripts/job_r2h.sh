#!/bin/bash
# fused4 register diet: x-factor rows + gather descriptors in LDS (default
# build, 2 waves/SIMD) and the same at 3 waves/SIMD (variant f4w3, 168 VGPRs,
# no spill); correctness of both, then an interleaved same-box A/B vs the old
# register layout (variant f4old).
source scripts/gpu_steps.sh
K="fused4 or version4 or -4- or golden or fused_cg_matches or segments"
step pytest_f4_new 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_runtime.py -q -rf --timeout 240 --timeout-method thread -k "$K"
BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_f4w3.so step pytest_f4_w3 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_runtime.py -q -rf --timeout 240 --timeout-method thread -k "$K"
CFGS=q3 VARIANTS="f4old new f4w3" REPS=3 BENCH_EXTRA="--extras off --profile-steps 0" bash scripts/job_abvar.sh
