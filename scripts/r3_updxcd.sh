#!/bin/bash
# Tiled r update with the XCD-aware block remap (prod) vs HEAD (prev).
source scripts/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step ux_tests 600 python -u -m pytest tests/test_gpu_runtime.py -x -q --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/ux_tests.log && ! grep -q "failed" gpurun_out/ux_tests.log || exit 1
for c in q3 q6 q6f32; do
  bash scripts/r3_ab.sh "--config $c --steps 100 --warmup 10 --companions off --extras off" prev
done
