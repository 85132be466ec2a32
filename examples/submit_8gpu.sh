#!/bin/bash
# One node, 8x MI355X, one process per GPU over RCCL/xGMI (analogue of the
# reference's examples/submit.sh, 16 nodes x 4 GH200 under SLURM/MPI).
set -e
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
RUN="python -m torch.distributed.run --nnodes=1 --nproc-per-node=8 --master-addr=127.0.0.1 --master-port=29500"
# correctness against the assembled matrix (reference: mat_comp-16.json)
$RUN -m benchmark_dolfinx_amd --nreps=1 --mat_comp --ndofs_global=100000 --degree=3 --json mat_comp-8.json
# headline runs: 300 M Q3 / 500 M Q6 DoFs per GPU, CG x 1000
$RUN -m benchmark_dolfinx_amd --ndofs=300000000 --degree=3 --cg --json Q3-300M.json
$RUN -m benchmark_dolfinx_amd --ndofs=500000000 --degree=6 --cg --json Q6-500M.json
# BASELINE.json config 5: Q6 500 M DoFs/GPU in FP32 on 8 GPUs
$RUN -m benchmark_dolfinx_amd --ndofs=500000000 --degree=6 --cg --float=32 --json Q6-500M-fp32.json
$RUN bench.py --gpus 8 --config q6f32
# weak-scaling curve of bench.py (1/2/4/8 GPUs)
for n in 1 2 4 8; do
  python -m torch.distributed.run --nnodes=1 --nproc-per-node=$n --master-addr=127.0.0.1 \
    --master-port=$((29600 + n)) bench.py --gpus $n --config q3
done
