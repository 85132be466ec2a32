#!/bin/bash
# PMC passes of one bench config, one counter group per rocprofv3 run (the
# box refuses groups over the per-block limits and --pmc with tracing).
#   bash scripts/pmc.sh TAG "<bench args>" [lib]
# lib: a libbdx_hip_NAME.so variant (same-box A/B), default the production build
source scripts/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; args=$2; lib=${3:-}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU GRBM_GUI_ACTIVE"
P3="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"
# FETCH_SIZE takes 3 of the 4 TCC slots and WRITE_SIZE 2: one pass each
P4="FETCH_SIZE"
P5="WRITE_SIZE"
if [ -n "$lib" ]; then
  export BDX_HIP_LIB=benchmark_dolfinx_amd/ops/libbdx_hip_$lib.so BDX_ALLOW_VARIANT=1
fi
passes=${PMC_PASSES:-1 2 3 4 5}
for pass in $passes; do
  eval "ctrs=\$P$pass"
  step pmc_${tag}_$pass 180 timeout -s KILL 170 rocprofv3 --pmc $ctrs --output-format csv \
    -d gpurun_out/pmc_${tag}/p$pass -o pmc -- python3 bench.py $args --companions off --extras off --profile-steps 0
done
