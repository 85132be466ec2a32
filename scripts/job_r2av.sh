#!/bin/bash
# fused3 x-trilinear instance (AFF = 2) on the reference's perturbed meshes:
# smoke, numerics against the CPU operator, then perturbed-mesh benches (auto
# = x-trilinear vs forced general trilinear), Q3 / Q6 FP64 and Q6 FP32.
source scripts/gpu_steps.sh
step xt_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step xt_pytest 600 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gpu_fused.py -m gpu -k "x_trilinear or fused3 or otf-3- or otf-2-"
for c in q3 q6 q6f32; do
  step xt_bench_${c}_auto 300 python -u bench.py --config $c --perturb 0.1 --extras off
  step xt_bench_${c}_gen 300 python -u bench.py --config $c --perturb 0.1 --geometry otf-general --extras off
done
