#!/bin/bash
# Round 3: dofmap kernel rewrite (line-per-lane, fused CG) + new two-stream
# schedule: GPU tests first, then benches, rehearsal and traces.
source scripts/gpu_steps.sh
step d_pytest_dofmap 300 python -u -m pytest tests/test_gpu_dofmap.py -q -x --timeout 120 --timeout-method thread
step d_pytest_gpu 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
step d_bench_dofmap 300 python -u bench.py --config q3 --kernel dofmap --geometry stored --steps 50 --warmup 5 --extras off --companions off
step d_bench_dofmap_otf 300 python -u bench.py --config q3 --kernel dofmap --steps 30 --warmup 3 --extras off --companions off
for i in 1 2; do
  for g in 0 1; do
    step s_graph${g}_$i 300 env BDX_GRAPH=$g python -u bench.py --steps 100 --warmup 10 --companions off --extras off
  done
done
step s_rehearse8 600 python -u scripts/fullsize_multirank.py --config q3 --per-rank 37500000 --ranks 8 --ref-ranks 1 --steps 10
step d_prof_dofmap 400 bash scripts/r3_prof_dofmap.sh
step ab_q6 600 bash scripts/r3_ab.sh "--config q6 --steps 100 --warmup 10 --companions off --extras off" f5w3
step ab_q6f32 600 bash scripts/r3_ab.sh "--config q6f32 --steps 100 --warmup 10 --companions off --extras off" f5w3
