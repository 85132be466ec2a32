#!/bin/bash
# Round 3: fused3 peeled accumulators (production) vs HEAD build, plus the
# GPU suite on the production build.
source scripts/gpu_steps.sh
step pl_pytest 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
bash scripts/r3_ab.sh "--config q3 --perturb 0.1 --geometry otf-general --steps 30 --warmup 3 --companions off --extras off" prev
bash scripts/r3_ab.sh "--config q3 --perturb 0.1 --steps 30 --warmup 3 --companions off --extras off" prev
bash scripts/r3_ab.sh "--config q6f32 --perturb 0.1 --steps 30 --warmup 3 --companions off --extras off" prev
