#!/bin/bash
# Round 3: new two-stream schedule (boundary tiles on the comm stream) under
# the GPU suite and an 8-rank threaded rehearsal; eager vs graph replay at
# N = 1; dofmap kernel trace.
source scripts/gpu_steps.sh
step s_pytest_gpu 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
for i in 1 2; do
  for g in 0 1; do
    step s_graph${g}_$i 300 env BDX_GRAPH=$g python -u bench.py --steps 100 --warmup 10 --companions off --extras off
  done
done
step s_rehearse8 600 python -u scripts/fullsize_multirank.py --config q3 --per-rank 37500000 --ranks 8 --ref-ranks 1 --steps 10
step s_prof_dofmap 400 bash scripts/r3_prof_dofmap.sh
