#!/bin/bash
# dofmap: 3 waves/SIMD build (w3, 25-VGPR spill) vs production; on-the-fly
# geometry on the same data model for comparison.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash scripts/r3_ab.sh "--config q3 --kernel dofmap --geometry stored --steps 30 --warmup 3 --companions off --extras off" w3
bash scripts/r3_ab.sh "--config q3 --kernel dofmap --geometry otf --steps 30 --warmup 3 --companions off --extras off"
bash scripts/r3_ab.sh "--config q3 --kernel dofmap --geometry otf --perturb 0.1 --steps 30 --warmup 3 --companions off --extras off"
