#!/bin/bash
# Evidence on the x-trilinear tree: GPU suite, smoke, default bench (with the
# random-kappa / x-trilinear / general-trilinear variants), kernel trace of the
# perturbed Q3 path, and the x-loop unroll A/B of the AFF = 2 instance.
source scripts/gpu_steps.sh
step aw_pytest_gpu 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
step aw_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step aw_bench_default 600 python -u bench.py
step aw_prof_q3pert 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/aw_prof_q3pert -o trace -- python3 bench.py --steps 20 --warmup 2 --perturb 0.1 --extras off
CFGS="q3 q6 q6f32" VARIANTS="new xq1" REPS=2 BENCH_EXTRA="--perturb 0.1 --extras off" bash scripts/job_abvar.sh
