#!/bin/bash
# Final check of the committed tree: GPU suite, smoke, the driver's bench
# command and the default bench.
source scripts/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step f3_pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step f3_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step f3_driver 400 python -u bench.py --gpus 1 --steps 20 --warmup 5
step f3_default 600 python -u bench.py
