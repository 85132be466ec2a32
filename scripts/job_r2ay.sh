#!/bin/bash
# Perturbed meshes: fused2 vs fused3 x-trilinear instances (qmode=1), and the
# qmode=0 (GLL collocation, fused2) x-trilinear vs general instance via the CLI.
source scripts/gpu_steps.sh
for c in q3 q6; do
  for rep in 1 2; do
    step ay_${c}_f3_$rep 300 python -u bench.py --config $c --perturb 0.1 --extras off --steps 100 --warmup 5
    step ay_${c}_f2_$rep 300 python -u bench.py --config $c --perturb 0.1 --extras off --steps 100 --warmup 5 --kernel fused2
  done
done
step ay_cli_q0_xt 300 python -u -m benchmark_dolfinx_amd --ndofs=300000000 --degree=3 --qmode=0 --cg --nreps=100 --geom_perturb_fact=0.1 --json gpurun_out/ay_q0_xt.json
step ay_cli_q0_gen 300 python -u -m benchmark_dolfinx_amd --ndofs=300000000 --degree=3 --qmode=0 --cg --nreps=100 --geom_perturb_fact=0.1 --geometry otf-general --json gpurun_out/ay_q0_gen.json
