#!/bin/bash
# fused4 prefetch depth 2: correctness, then a same-box A/B vs depth 1
source scripts/gpu_steps.sh
step pytest_f4 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_runtime.py -q -rf --timeout 240 --timeout-method thread -k "fused4 or version4 or 4-3 or -4- or golden or runtime or overlap or segments"
step q3_d1 200 env BDX_F4_DEPTH=1 python bench.py --steps 30 --warmup 5 --profile-steps 0
step q3_d2 200 env BDX_F4_DEPTH=2 python bench.py --steps 30 --warmup 5
step q3_d1b 200 env BDX_F4_DEPTH=1 python bench.py --steps 30 --warmup 5 --profile-steps 0
step q3_d2b 200 env BDX_F4_DEPTH=2 python bench.py --steps 30 --warmup 5 --profile-steps 0
step q3_d2_rk 200 env BDX_F4_DEPTH=2 python bench.py --steps 30 --warmup 5 --profile-steps 0 --kappa random
