#!/bin/bash
# Runtime suite after the fused3 tiled opt-in (BDX_TILED=2) and alignment gate.
source scripts/gpu_steps.sh
step t_rt 700 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_runtime.py -m gpu
