#!/bin/bash
# Tiled r update, row-vector form: GPU suite, then A/B against HEAD (prev) on
# the three headline configs.
source scripts/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step upd_pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/upd_pytest.log && ! grep -q "failed" gpurun_out/upd_pytest.log || exit 1
for c in q3 q6 q6f32; do
  bash scripts/r3_ab.sh "--config $c --steps 100 --warmup 10 --companions off --extras off" prev
done
