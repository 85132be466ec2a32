#!/bin/bash
# Q6 FP64 perturbed (fused3 x-trilinear): output-descriptor recomputation
# (203 vs 234 VGPRs, both 2 waves/SIMD) and forced x-segment counts vs auto.
source scripts/gpu_steps.sh
for rep in 1 2; do
  step bb_auto_$rep 300 python -u bench.py --config q6 --perturb 0.1 --extras off --steps 100 --warmup 5
  BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_xor.so step bb_xor_$rep 300 python -u bench.py --config q6 --perturb 0.1 --extras off --steps 100 --warmup 5
  for s in 1 2 4; do
    BDX_SEGMENTS=$s step bb_seg${s}_$rep 300 python -u bench.py --config q6 --perturb 0.1 --extras off --steps 100 --warmup 5
  done
done
