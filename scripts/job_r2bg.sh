#!/bin/bash
# Kernel tables of the box headline configs on the final tree (segment model).
source scripts/gpu_steps.sh
for c in q3 q6; do
  step bg_prof_$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bg_prof_$c -o trace -- python3 bench.py --config $c --steps 20 --warmup 2 --profile-steps 0 --extras off
done
