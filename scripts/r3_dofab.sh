#!/bin/bash
# Round 3: dofmap kernel A/B (production vs HEAD build vs 3-wave variant),
# after the dofmap GPU tests on the production build.
source scripts/gpu_steps.sh
step dof_tests 600 python -u -m pytest tests/test_gpu_dofmap.py -q -x --timeout 120 --timeout-method thread
bash scripts/r3_ab.sh "--config q3 --kernel dofmap --geometry stored --steps 30 --warmup 3 --companions off --extras off" prev w3
