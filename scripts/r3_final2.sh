#!/bin/bash
# Round-3 final evidence (re-entry session): GPU suite, smoke, the driver's
# bench command, the default bench, kernel traces of the headline configs and
# the dofmap data model.
source scripts/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step f2_pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step f2_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step f2_driver 400 python -u bench.py --gpus 1 --steps 20 --warmup 5
step f2_default 600 python -u bench.py
for c in q3 q6 q6f32; do
  step f2_trace_$c 240 rocprofv3 --kernel-trace --stats -d gpurun_out/f2_trace_$c -o run -- python3 bench.py --config $c --steps 30 --warmup 3 --companions off --extras off --profile-steps 0
done
step f2_trace_dofmap 240 rocprofv3 --kernel-trace --stats -d gpurun_out/f2_trace_dofmap -o run -- python3 bench.py --config q3 --kernel dofmap --geometry stored --steps 20 --warmup 3 --companions off --extras off --profile-steps 0
