#!/bin/bash
# rocprofv3 kernel traces (--kernel-trace --stats only) of bench configs,
# summarised on the box (scripts/prof_db.py -> gpurun_out/tr_TAG_i.txt) and the
# databases deleted, so the copy-back stays small.
#   bash scripts/trace.sh TAG "<bench args>" ["<bench args>" ...]
# e.g. bash scripts/trace.sh q3 "--config q3 --steps 30 --warmup 3"
source scripts/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; shift
i=0
for args in "$@"; do
  d=gpurun_out/tr_${tag}_$i
  step tr_${tag}_$i 300 rocprofv3 --kernel-trace --stats -d $d -o run -- \
    python3 bench.py $args --companions off --extras off --profile-steps 0
  { echo "== $args"; for db in $(find $d -name '*.db'); do python3 scripts/prof_db.py $db --top 12; done; } \
    > gpurun_out/tr_${tag}_$i.txt
  rm -rf $d
  i=$((i + 1))
done
