#!/bin/bash
# Round 3: dofmap kernel (pipelined) -- tests, bench, trace; 8-rank rehearsal timeline.
source scripts/gpu_steps.sh
step d2_pytest_dofmap 300 python -u -m pytest tests/test_gpu_dofmap.py -q -x --timeout 120 --timeout-method thread
step d2_bench_dofmap 300 python -u bench.py --config q3 --kernel dofmap --geometry stored --steps 50 --warmup 5 --extras off --companions off
step d2_bench_dofmap_otf 300 python -u bench.py --config q3 --kernel dofmap --steps 30 --warmup 3 --extras off --companions off
step d2_rehearse8 600 python -u scripts/fullsize_multirank.py --config q3 --per-rank 37500000 --ranks 8 --ref-ranks 1 --steps 10
mkdir -p gpurun_out/r3prof2
step d2_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3prof2/dofmap -o run -- python3 bench.py --config q3 --kernel dofmap --geometry stored --steps 20 --warmup 3 --extras off --companions off --profile-steps 0
