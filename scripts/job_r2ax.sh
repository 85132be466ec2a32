#!/bin/bash
# Overlap evidence: runtime phase tests, then the 8-rank (1x2x4) geometry of
# the driver's N = 8 run as threaded ranks on one GPU (37.5 M Q3 DoFs per rank)
# against 4 ranks; rank phases carry the forward/reverse exchange completion
# times against the interior-tile completion times.
source scripts/gpu_steps.sh
step ax_pytest_rt 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gpu_runtime.py -m gpu
step ax_rehearse_q3 600 python -u scripts/fullsize_multirank.py --config q3 --per-rank 37500000 --ranks 8 --ref-ranks 4 --steps 20
