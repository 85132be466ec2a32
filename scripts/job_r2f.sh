#!/bin/bash
# Round-2 evidence pass on the rebuilt tree: GPU suite, smoke, fused4 prefetch
# depth A/B, the other headline configs, and a kernel-trace profile of Q3.
source scripts/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step q3_d1 200 env BDX_F4_DEPTH=1 python bench.py --steps 30 --warmup 5 --profile-steps 0
step q3_d2 200 env BDX_F4_DEPTH=2 python bench.py --steps 30 --warmup 5
step q3_d1b 200 env BDX_F4_DEPTH=1 python bench.py --steps 30 --warmup 5 --profile-steps 0
step q3_d2b 200 env BDX_F4_DEPTH=2 python bench.py --steps 30 --warmup 5 --profile-steps 0
step q3_rk 200 python bench.py --steps 30 --warmup 5 --kappa random
step q6 300 python bench.py --config q6 --steps 20 --warmup 5
step q6f32 300 python bench.py --config q6f32 --steps 20 --warmup 5
step q3gen 300 python bench.py --perturb 0.1 --steps 20 --warmup 5
step trace_q3 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_q3 -o trace -- python3 bench.py --steps 20 --warmup 2 --profile-steps 0
