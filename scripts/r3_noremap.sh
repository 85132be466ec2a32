#!/bin/bash
# XCD-aware block remap vs launch order (no remap) in the operator kernels:
# fused5 (f5norm), dofmap (dofnorm), fused3 (f3norm); same box, interleaved.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in q3 q6 q6f32; do
  bash scripts/r3_ab.sh "--config $c --steps 100 --warmup 10 --companions off --extras off" f5norm
done
bash scripts/r3_ab.sh "--config q3 --kernel dofmap --geometry stored --steps 30 --warmup 3 --companions off --extras off" dofnorm
bash scripts/r3_ab.sh "--config q3 --perturb 0.1 --steps 50 --warmup 5 --companions off --extras off" f3norm
