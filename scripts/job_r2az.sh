#!/bin/bash
# x-trilinear fused3 on tile-major CG storage (BDX_TILED=2) vs the lattice
# layout, perturbed Q3 / Q6 FP64 / Q6 FP32, interleaved.
source scripts/gpu_steps.sh
for c in q3 q6 q6f32; do
  for rep in 1 2; do
    step az_${c}_lat_$rep 300 python -u bench.py --config $c --perturb 0.1 --extras off --steps 100 --warmup 5
    BDX_TILED=2 step az_${c}_til_$rep 300 python -u bench.py --config $c --perturb 0.1 --extras off --steps 100 --warmup 5
  done
done
