#!/bin/bash
# Tiled r update with the next grid-stride step's loads in flight (pipe) vs
# production: runtime tests, then A/B on the three headline configs.
source scripts/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step up_tests 600 env BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_pipe.so BDX_ALLOW_VARIANT=1 python -u -m pytest tests/test_gpu_runtime.py -x -q -k "not test_bench_entry_point_one_gpu" --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/up_tests.log && ! grep -q "failed" gpurun_out/up_tests.log || exit 1
for c in q3 q6 q6f32; do
  bash scripts/r3_ab.sh "--config $c --steps 100 --warmup 10 --companions off --extras off" pipe
done
