#!/bin/bash
# Full-size CG iterate pin (Q3 300 M: fused5 and fused4; Q6 500 M: fused5) vs the stored-G v1 kernel.
source scripts/gpu_steps.sh
step fullsize_pin 900 python -u -m pytest -v -s --timeout 400 --timeout-method thread tests/test_gpu_fullsize_cg.py -m gpu
