#!/bin/bash
# Full-size single-GPU runs through the reference's command line (one GPU's
# share of the reference's headline runs); the JSONs are the committed
# examples/mi355x/*.json (tests/test_fullsize_examples.py pins them).
#   bash scripts/job_fullsize.sh [outdir]     (default gpurun_out/fullsize)
source scripts/gpu_steps.sh
out=${1:-gpurun_out/fullsize}
mkdir -p "$out"
step fs_q3 300 python -u -m benchmark_dolfinx_amd --degree=3 --ndofs=300000000 --cg --nreps=1000 --json "$out/Q3-300M.json"
step fs_q6 300 python -u -m benchmark_dolfinx_amd --degree=6 --ndofs=500000000 --cg --nreps=1000 --json "$out/Q6-500M.json"
step fs_q6f32 300 python -u -m benchmark_dolfinx_amd --degree=6 --ndofs=500000000 --cg --nreps=1000 --float=32 --json "$out/Q6-500M-fp32.json"
step fs_q3a 300 python -u -m benchmark_dolfinx_amd --degree=3 --ndofs=300000000 --nreps=200 --json "$out/Q3-300M-action.json"
step fs_q6a 300 python -u -m benchmark_dolfinx_amd --degree=6 --ndofs=500000000 --nreps=200 --json "$out/Q6-500M-action.json"
