#!/bin/bash
# Round 3: PMC passes (one counter group per rocprofv3 run) for Q6 FP64 /
# FP32 fused5 and the Q3 dofmap kernel.
source scripts/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU GRBM_GUI_ACTIVE"
for cfg in "q6:--config q6" "q6f32:--config q6f32" "dof:--config q3 --kernel dofmap --geometry stored"; do
  name=${cfg%%:*}; args=${cfg#*:}
  for pass in 1 2; do
    eval "ctrs=\$P$pass"
    step pmc_${name}_$pass 120 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/pmc/$name$pass -o pmc -- python3 bench.py $args --steps 10 --warmup 2 --companions off --extras off --profile-steps 0
  done
done
