#!/bin/bash
# GPU suite (incl. determinism tests), then the kernel tests against the
# BDX_DEBUG build (device-side index checks) of the HIP library.
source scripts/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread
BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_debug.so step pytest_debug 900 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_dofmap.py tests/test_gpu_runtime.py tests/test_gpu_determinism.py -q -rf --timeout 240 --timeout-method thread
BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_debug.so step bench_debug 300 python -u bench.py --steps 5 --warmup 1 --extras off --profile-steps 0
