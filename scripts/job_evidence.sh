#!/bin/bash
# Round evidence on the committed tree: GPU suite, smoke, headline benches,
# rocprofv3 kernel tables (Q3 fused4, Q6 fused5, Q6-FP32 fused5).
source scripts/gpu_steps.sh
step ev_pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
step ev_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step ev_bench_default 600 python -u bench.py
step ev_bench_q6 600 python -u bench.py --config q6
step ev_bench_q6f32 600 python -u bench.py --config q6f32
step ev_bench_q3_random 600 python -u bench.py --kappa random
for c in q3 q6 q6f32; do
  step ev_prof_$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ev_prof_$c -o trace -- python3 bench.py --steps 20 --warmup 2 --config $c
done
