#!/bin/bash
# dofmap: next-cell gathers + stored G issued right after the F stage (prod)
# vs at the end of the cell (prev = HEAD), and prod with non-temporal G loads (nt).
source scripts/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step dof_tests 600 python -u -m pytest tests/test_gpu_dofmap.py -q -x --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/dof_tests.log && ! grep -q "failed" gpurun_out/dof_tests.log || exit 1
bash scripts/r3_ab.sh "--config q3 --kernel dofmap --geometry stored --steps 30 --warmup 3 --companions off --extras off" prev nt
bash scripts/r3_ab.sh "--config q6 --kernel dofmap --geometry stored --steps 10 --warmup 2 --companions off --extras off" prev
