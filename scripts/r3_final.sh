#!/bin/bash
# Round 3 final evidence on one box: smoke, the driver's bench command, the
# default bench, and rocprofv3 kernel traces of the Q3 / Q6 / Q6-FP32
# headline configs (summaries: scripts/prof_db.py).
source scripts/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step fin_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step fin_driver 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step fin_default 600 python -u bench.py
for c in q3 q6 q6f32; do
  step fin_trace_$c 240 rocprofv3 --kernel-trace --stats -d gpurun_out/fin_trace_$c -o run -- python3 bench.py --config $c --steps 30 --warmup 3 --companions off --extras off --profile-steps 0
done
