#!/bin/bash
# Per-step device times of the driver's command (twice) and of a 200-step run
# in one call: is the 20-step window slower than steady state on this box?
source scripts/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step st_a 300 env BDX_STEP_TRACE=gpurun_out/steps_a.jsonl python -u bench.py --gpus 1 --steps 20 --warmup 5 --companions off --extras off
step st_b 300 env BDX_STEP_TRACE=gpurun_out/steps_b.jsonl python -u bench.py --gpus 1 --steps 200 --warmup 5 --companions off --extras off
step st_c 300 env BDX_STEP_TRACE=gpurun_out/steps_c.jsonl python -u bench.py --gpus 1 --steps 20 --warmup 5 --companions off --extras off
