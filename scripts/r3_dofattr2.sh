#!/bin/bash
# Attribution of the element-role dofmap kernel: timing-only variants that
# drop the scatter atomics (na), the stored-G loads (ng), the r / p_old / x
# gathers (ngat) or all three (nall); wrong numerics, same box, interleaved.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash scripts/r3_ab.sh "--config q3 --kernel dofmap --geometry stored --steps 30 --warmup 3 --companions off --extras off --profile-steps 3" na ng ngat nall
