#!/bin/bash
# Round-3 evidence on the tree after the dofmap element role and the FP32
# row-vector update: GPU suite, smoke, the driver's bench command, the default
# bench, and kernel traces of the dofmap and Q6 FP32 configurations.
source scripts/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step ev_pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step ev_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step ev_driver 400 python -u bench.py --gpus 1 --steps 20 --warmup 5
step ev_default 600 python -u bench.py
step ev_trace_dofmap 240 rocprofv3 --kernel-trace --stats -d gpurun_out/ev_trace_dofmap -o run -- python3 bench.py --config q3 --kernel dofmap --geometry stored --steps 20 --warmup 3 --companions off --extras off --profile-steps 0
step ev_trace_q6f32 240 rocprofv3 --kernel-trace --stats -d gpurun_out/ev_trace_q6f32 -o run -- python3 bench.py --config q6f32 --steps 30 --warmup 3 --companions off --extras off --profile-steps 0
