#!/bin/bash
# Full-size single-GPU runs of the reference's headline configurations through
# the CLI (the bench_dolfinx command line), JSON kept for examples/mi355x/.
source scripts/gpu_steps.sh
mkdir -p gpurun_out/fullsize
C="python -u -m benchmark_dolfinx_amd --platform=gpu --qmode=1"
step fs_q3_action 300 $C --ndofs=300000000 --degree=3 --float=64 --nreps=200 --json gpurun_out/fullsize/Q3-300M-action.json
step fs_q3_cg 300 $C --ndofs=300000000 --degree=3 --float=64 --cg --nreps=1000 --json gpurun_out/fullsize/Q3-300M.json
step fs_q6_action 300 $C --ndofs=500000000 --degree=6 --float=64 --nreps=200 --json gpurun_out/fullsize/Q6-500M-action.json
step fs_q6_cg 300 $C --ndofs=500000000 --degree=6 --float=64 --cg --nreps=1000 --json gpurun_out/fullsize/Q6-500M.json
step fs_q6f32_cg 300 $C --ndofs=500000000 --degree=6 --float=32 --cg --nreps=1000 --json gpurun_out/fullsize/Q6-500M-fp32.json
