#!/bin/bash
# Round-end style check of the current tree on a GPU box: the GPU suite, the
# driver's smoke, the driver's bench command and the default bench.
#   bash scripts/check_tree.sh TAG [extra pytest args]
source scripts/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-check}; shift
step ${tag}_pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "$@"
step ${tag}_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step ${tag}_driver 400 python -u bench.py --gpus 1 --steps 20 --warmup 5
step ${tag}_default 600 python -u bench.py
