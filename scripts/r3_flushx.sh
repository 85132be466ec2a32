#!/bin/bash
# Round 3: fused flush + export at the end of a CG call: GPU suite, then the
# driver's 20-step command and a 200-step run, production vs HEAD build; and
# fused3 with peeled accumulator initialisation (variant "peel").
source scripts/gpu_steps.sh
step fx_pytest 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
bash scripts/r3_ab.sh "--gpus 1 --steps 20 --warmup 5 --companions off --extras off" prev
bash scripts/r3_ab.sh "--gpus 1 --steps 200 --warmup 10 --companions off --extras off" prev
bash scripts/r3_ab.sh "--config q3 --perturb 0.1 --steps 30 --warmup 3 --companions off --extras off" peel
bash scripts/r3_ab.sh "--config q6 --perturb 0.1 --steps 30 --warmup 3 --companions off --extras off" peel
bash scripts/r3_ab.sh "--config q3 --perturb 0.1 --geometry otf-general --steps 30 --warmup 3 --companions off --extras off" peel
