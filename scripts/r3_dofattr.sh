#!/bin/bash
# Round 3: dofmap phase attribution (timing-only variant builds, wrong
# numerics): na = no scatter atomics, ng = no stored-G loads, ngat = no dof
# value gathers, nall = all three removed (compute + dofmap/flag loads only).
source scripts/gpu_steps.sh
rm -f gpurun_out/ab_summary.txt
bash scripts/r3_ab.sh "--config q3 --kernel dofmap --geometry stored --steps 30 --warmup 3 --companions off --extras off --profile-steps 3" na ng ngat nall
