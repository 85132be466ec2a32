#!/bin/bash
# fused4 x segments: correctness, then a same-box A/B (whole-x vs auto segments)
source scripts/gpu_steps.sh
step pytest_seg 600 python -u -m pytest tests/test_gpu_fused.py -q -rf --timeout 240 --timeout-method thread -k "segments or golden or fused_cg_matches or partition_invariance_threaded"
step q3_seg1 200 env BDX_SEGMENTS=1 python bench.py --steps 30 --warmup 5 --profile-steps 0
step q3_auto 200 python bench.py --steps 30 --warmup 5 --profile-steps 0
step q3_seg1b 200 env BDX_SEGMENTS=1 python bench.py --steps 30 --warmup 5 --profile-steps 0
step q3_autob 200 python bench.py --steps 30 --warmup 5
step q3_seg4 200 env BDX_SEGMENTS=4 python bench.py --steps 30 --warmup 5 --profile-steps 0
step q3_seg8 200 env BDX_SEGMENTS=8 python bench.py --steps 30 --warmup 5 --profile-steps 0
