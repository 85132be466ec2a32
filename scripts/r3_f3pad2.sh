#!/bin/bash
# fused3 Q3 padding: isolate the slowdown (padded lanes with the block layout
# = padblock; padded wave-local with a 2 x 4 tile = tile24) against prod
# (padded, wave-local, 2 x 5) and HEAD (prev).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash scripts/r3_ab.sh "--config q3 --perturb 0.1 --steps 30 --warmup 3 --companions off --extras off" prev padblock tile24
