#!/bin/bash
# Round-3 re-entry: GPU suite, smoke and the driver's bench command on the
# working tree, then the dofmap scatter A/B against HEAD's library (prev).
source scripts/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step head_pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step head_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step head_driver 400 python -u bench.py --gpus 1 --steps 20 --warmup 5
bash scripts/r3_ab.sh "--config q3 --kernel dofmap --geometry stored --steps 30 --warmup 3 --companions off --extras off" prev
