#!/bin/bash
# PMC pass of the padded (prod) vs unpadded (prev) fused3 Q3 x-trilinear kernel.
source scripts/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVES"
step pmc_pad 120 rocprofv3 --pmc $P2 --output-format csv -d gpurun_out/pmcpad/prod -o pmc -- python3 bench.py --config q3 --perturb 0.1 --steps 6 --warmup 2 --companions off --extras off --profile-steps 0
step pmc_prev 120 env BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_prev.so BDX_ALLOW_VARIANT=1 rocprofv3 --pmc $P2 --output-format csv -d gpurun_out/pmcpad/prev -o pmc -- python3 bench.py --config q3 --perturb 0.1 --steps 6 --warmup 2 --companions off --extras off --profile-steps 0
