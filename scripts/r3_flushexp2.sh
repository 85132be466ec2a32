#!/bin/bash
# flush_export staged through LDS per (x, tile row, z group): GPU suite, kernel
# traces, and the driver's 20-step shape against HEAD (prev).
source scripts/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step fe2_pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/fe2_pytest.log && ! grep -q "failed" gpurun_out/fe2_pytest.log || exit 1
for c in q3 q6 q6f32; do
  step fe2_trace_$c 240 rocprofv3 --kernel-trace --stats -d gpurun_out/fe2_trace_$c -o run -- python3 bench.py --config $c --steps 20 --warmup 5 --companions off --extras off --profile-steps 0
done
for c in q3 q6; do
  bash scripts/r3_ab.sh "--config $c --steps 20 --warmup 5 --companions off --extras off" prev
done
