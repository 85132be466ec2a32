#!/bin/bash
# Runtime tests after the test fix + tail-effect probe of fused4: the same
# DoF count with a (y, z) tile grid of exactly 6 rounds (48 x 64 tiles = 3072
# = 6 x 512 resident workgroups) vs the default 56 x 56 = 3136 (6.1 rounds).
source scripts/gpu_steps.sh
step pytest_rt 600 python -u -m pytest tests/test_gpu_runtime.py -q -rf --timeout 240 --timeout-method thread
step tail_3136 200 python bench.py --steps 30 --warmup 5 --profile-steps 0 --mesh 222,223,223
step tail_3072 200 python bench.py --steps 30 --warmup 5 --profile-steps 0 --mesh 258,192,256
step tail_3584 200 python bench.py --steps 30 --warmup 5 --profile-steps 0 --mesh 193,224,256
step tail_3136b 200 python bench.py --steps 30 --warmup 5 --profile-steps 0 --mesh 222,223,223
