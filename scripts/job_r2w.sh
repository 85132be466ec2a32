#!/bin/bash
# Release-build GPU suite (kernels serialized so that a fault names its
# kernel), stop at the first failure.
source scripts/gpu_steps.sh
AMD_SERIALIZE_KERNEL=3 step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 240 --timeout-method thread
