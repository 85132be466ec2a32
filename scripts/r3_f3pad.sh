#!/bin/bash
# fused3 Q3: 25 quadrature columns padded to 32 lanes (two cells per wave,
# wave-local intra-cell syncs) vs HEAD (prev): fused tests, then same-box A/B
# on the perturbed mesh (x-trilinear instance) and forced general geometry.
source scripts/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step f3_tests 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_runtime.py -q -x --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/f3_tests.log && ! grep -q "failed" gpurun_out/f3_tests.log || exit 1
bash scripts/r3_ab.sh "--config q3 --perturb 0.1 --steps 50 --warmup 5 --companions off --extras off" prev
bash scripts/r3_ab.sh "--config q3 --perturb 0.1 --geometry otf-general --steps 50 --warmup 5 --companions off --extras off" prev
