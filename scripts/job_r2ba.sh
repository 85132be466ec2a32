#!/bin/bash
# Evidence on the final round-2 tree: GPU suite, smoke, default bench (with
# variants), perturbed Q3 / Q6 / Q6-FP32 benches, perturbed Q6 kernel trace.
source scripts/gpu_steps.sh
step ba_pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
step ba_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step ba_bench_default 600 python -u bench.py
for c in q6 q6f32; do
  step ba_bench_${c}_pert 300 python -u bench.py --config $c --perturb 0.1 --extras off
done
step ba_prof_q6pert 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ba_prof_q6pert -o trace -- python3 bench.py --config q6 --steps 20 --warmup 2 --perturb 0.1 --extras off
