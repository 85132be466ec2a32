#!/bin/bash
# x-segment count A/B for the fused5 headline configs (box mesh), interleaved
# with the auto choice.
source scripts/gpu_steps.sh
for rep in 1 2; do
  for c in q6 q3 q6f32; do
    step bd_${c}_auto_$rep 300 python -u bench.py --config $c --extras off --steps 100 --warmup 5
    for s in 1 2 3 4; do
      BDX_SEGMENTS=$s step bd_${c}_seg${s}_$rep 300 python -u bench.py --config $c --extras off --steps 100 --warmup 5
    done
  done
done
