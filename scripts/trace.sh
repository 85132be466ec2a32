#!/bin/bash
# rocprofv3 kernel traces (--kernel-trace --stats only) of bench configs.
#   bash scripts/trace.sh TAG "<bench args>" ["<bench args>" ...]
# e.g. bash scripts/trace.sh q3 "--config q3 --steps 30 --warmup 3"
source scripts/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; shift
i=0
for args in "$@"; do
  step tr_${tag}_$i 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_${tag}_$i -o run -- \
    python3 bench.py $args --companions off --extras off --profile-steps 0
  i=$((i + 1))
done
