#!/bin/bash
# flush_export in tiled order with 16-byte vectors vs HEAD (prev): GPU suite,
# the driver's 20-step command shape on Q3 / Q6 FP32, and a kernel trace.
source scripts/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step fe_pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/fe_pytest.log && ! grep -q "failed" gpurun_out/fe_pytest.log || exit 1
for c in q3 q6f32; do
  bash scripts/r3_ab.sh "--config $c --steps 20 --warmup 5 --companions off --extras off" prev
done
step fe_trace 240 rocprofv3 --kernel-trace --stats -d gpurun_out/fe_trace -o run -- python3 bench.py --config q3 --steps 20 --warmup 5 --companions off --extras off --profile-steps 0
