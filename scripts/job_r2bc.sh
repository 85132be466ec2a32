#!/bin/bash
# x-segment count A/B for fused3 x-trilinear (perturbed meshes), interleaved.
source scripts/gpu_steps.sh
for rep in 1 2; do
  for s in 1 2 3 4; do
    BDX_SEGMENTS=$s step bc_q3_seg${s}_$rep 300 python -u bench.py --config q3 --perturb 0.1 --extras off --steps 100 --warmup 5
    BDX_SEGMENTS=$s step bc_q6f32_seg${s}_$rep 300 python -u bench.py --config q6f32 --perturb 0.1 --extras off --steps 100 --warmup 5
  done
  for s in 1 2 3; do
    BDX_SEGMENTS=$s step bc_q6_seg${s}_$rep 300 python -u bench.py --config q6 --perturb 0.1 --extras off --steps 100 --warmup 5
  done
done
