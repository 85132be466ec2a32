#!/bin/bash
# Round 3: cold-start profile of the driver's bench command on a fresh box
# (per-step device times via BDX_STEP_TRACE), then the same command warm.
source scripts/gpu_steps.sh
export BDX_STEP_TRACE=gpurun_out/step_trace.jsonl
rm -f $BDX_STEP_TRACE
step cold_driver 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 $COLD_ARGS
step long_400 300 python -u bench.py --gpus 1 --steps 400 --warmup 0 --companions off --extras off --profile-steps 0
step warm_driver 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 $COLD_ARGS
