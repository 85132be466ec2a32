#!/bin/bash
# x segments in fused2/3/5: full GPU suite, then Q6 / Q6 FP32 / general-geometry A/B
source scripts/gpu_steps.sh
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread
step q6_seg1 200 env BDX_SEGMENTS=1 python bench.py --config q6 --steps 20 --warmup 5 --profile-steps 0
step q6_auto 200 python bench.py --config q6 --steps 20 --warmup 5
step q6f32_seg1 200 env BDX_SEGMENTS=1 python bench.py --config q6f32 --steps 20 --warmup 5 --profile-steps 0
step q6f32_auto 200 python bench.py --config q6f32 --steps 20 --warmup 5
step q3gen_seg1 300 env BDX_SEGMENTS=1 python bench.py --perturb 0.1 --steps 20 --warmup 5 --profile-steps 0
step q3gen_auto 300 python bench.py --perturb 0.1 --steps 20 --warmup 5
step q3_auto 200 python bench.py --steps 20 --warmup 5
