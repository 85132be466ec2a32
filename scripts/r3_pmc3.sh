#!/bin/bash
# Round 3: GPU suite re-check, then PMC passes (one counter group per
# rocprofv3 run) for the fused3 instances: Q3 / Q6 perturbed (x-trilinear)
# and Q3 forced general trilinear geometry.
source scripts/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step r3_pytest_gpu_final 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU GRBM_GUI_ACTIVE"
P3="SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_ADD_F64 SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_ACTIVE_INST_FLAT SQ_INSTS_VALU_FMA_F64 GRBM_COUNT"
for cfg in "q3p:--config q3 --perturb 0.1" "q6p:--config q6 --perturb 0.1" "q3g:--config q3 --perturb 0.1 --geometry otf-general"; do
  name=${cfg%%:*}; args=${cfg#*:}
  for pass in 1 2 3; do
    eval "ctrs=\$P$pass"
    step pmc3_${name}_$pass 120 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/pmc3/$name$pass -o pmc -- python3 bench.py $args --steps 10 --warmup 2 --companions off --extras off --profile-steps 0
  done
done
