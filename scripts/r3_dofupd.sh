#!/bin/bash
# dofmap CG update in 16-byte vectors vs HEAD (prev): dofmap tests, A/B, trace.
source scripts/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step du_tests 600 python -u -m pytest tests/test_gpu_dofmap.py -x -q --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/du_tests.log && ! grep -q "failed" gpurun_out/du_tests.log || exit 1
bash scripts/r3_ab.sh "--config q3 --kernel dofmap --geometry stored --steps 30 --warmup 3 --companions off --extras off" prev
step du_trace 240 rocprofv3 --kernel-trace --stats -d gpurun_out/du_trace -o run -- python3 bench.py --config q3 --kernel dofmap --geometry stored --steps 20 --warmup 3 --companions off --extras off --profile-steps 0
