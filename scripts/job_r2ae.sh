#!/bin/bash
# Evidence pass after the descriptor laundering / fused5-at-Q3 switch: GPU
# suite, smoke, the driver-style bench (defaults), Q6 / Q6-FP32, kernel traces.
source scripts/gpu_steps.sh
step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 600 python bench.py
step bench_q6 600 python bench.py --config q6 --steps 100 --warmup 10
step bench_q6f32 600 python bench.py --config q6f32 --steps 100 --warmup 10
step trace_q3 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_q3 -o trace -- python3 bench.py --steps 20 --warmup 2 --profile-steps 0 --extras off
step trace_q6 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_q6 -o trace -- python3 bench.py --config q6 --steps 20 --warmup 2 --profile-steps 0 --extras off
step trace_q6f32 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_q6f32 -o trace -- python3 bench.py --config q6f32 --steps 20 --warmup 2 --profile-steps 0 --extras off
