#!/bin/bash
# 8-rank partition rehearsal on one GPU (threaded ranks, RCCL rules emulated,
# native runtime, thread transport, tiled storage) against 4 ranks on the
# same global mesh, at half the driver's per-rank size (memory of 8 ranks on
# one card): production kernels (fused5) at Q3 and Q6.
source scripts/gpu_steps.sh
step mr_q3 600 python -u scripts/fullsize_multirank.py --config q3 --per-rank 150000000 --ranks 8 --ref-ranks 4 --steps 20
step mr_q6 600 python -u scripts/fullsize_multirank.py --config q6 --per-rank 250000000 --ranks 8 --ref-ranks 4 --steps 20
