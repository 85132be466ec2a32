#!/bin/bash
# dofmap: stored-G prefetch in registers (prod, 2 waves/SIMD) vs G loaded at
# use with 4 (nopref) or 5 (nopref5) waves/SIMD; same box, interleaved.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash scripts/r3_ab.sh "--config q3 --kernel dofmap --geometry stored --steps 30 --warmup 3 --companions off --extras off" nopref nopref5
