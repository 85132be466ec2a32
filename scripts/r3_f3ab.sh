#!/bin/bash
# Round 3: fused3 A/B: 2-way unrolled x loop (u2), LDS tables in the x loop (tl).
source scripts/gpu_steps.sh
rm -f gpurun_out/ab_summary.txt
for cfg in "--config q3 --perturb 0.1" "--config q3 --perturb 0.1 --geometry otf-general" "--config q6 --perturb 0.1"; do
  bash scripts/r3_ab.sh "$cfg --steps 30 --warmup 3 --companions off --extras off" u2 tl || exit $?
done
