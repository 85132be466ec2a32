#!/bin/bash
# Round 3: chunk-mapped r update -- GPU suite, then same-box A/B against the
# previous revision's library (prev) on Q3 / Q6 / Q6-FP32.
source scripts/gpu_steps.sh
step u_pytest_gpu 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
step u_ab_q3 600 bash scripts/r3_ab.sh "--config q3 --steps 100 --warmup 10 --companions off --extras off" prev
step u_ab_q6 600 bash scripts/r3_ab.sh "--config q6 --steps 100 --warmup 10 --companions off --extras off" prev
step u_ab_q6f32 600 bash scripts/r3_ab.sh "--config q6f32 --steps 100 --warmup 10 --companions off --extras off" prev
