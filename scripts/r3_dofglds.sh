#!/bin/bash
# dofmap stored G as 16-byte chunks redistributed through LDS (glds) vs
# production: dofmap tests, then A/B at Q3 (qmode 1) and Q2 / Q1.
source scripts/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step dg_tests 600 env BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_glds.so BDX_ALLOW_VARIANT=1 python -u -m pytest tests/test_gpu_dofmap.py -x -q --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/dg_tests.log && ! grep -q "failed" gpurun_out/dg_tests.log || exit 1
bash scripts/r3_ab.sh "--config q3 --kernel dofmap --geometry stored --steps 30 --warmup 3 --companions off --extras off" glds
