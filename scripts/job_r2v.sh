#!/bin/bash
# Memory-safety hunt: the GPU suite on the BDX_DEBUG library (bounds-checked
# global accesses in the fused kernels, tiled update and layout conversion:
# an out-of-range offset is printed and the access skipped).
source scripts/gpu_steps.sh
BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_debug.so step pytest_debug 900 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread -s -p no:randomly
grep -a "bdx OOB\|bdx ASSERT" gpurun_out/pytest_debug.log | sort | uniq -c | sort -rn | head -30 > gpurun_out/oob_summary.txt || true
