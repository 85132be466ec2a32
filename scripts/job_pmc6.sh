#!/bin/bash
# PMC passes on the laundered tree: fused5 (Q3, Q6 FP64, Q6 FP32) and fused3
# general (Q3 --perturb 0.1).  One counter group per run.
source scripts/gpu_steps.sh
P="rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc6"
for cfg in q3 q6 q6f32 q3g; do
  case $cfg in
    q3g) B="python3 bench.py --steps 3 --warmup 1 --config q3 --perturb 0.1 --extras off --profile-steps 0" ;;
    *) B="python3 bench.py --steps 3 --warmup 1 --config $cfg --extras off --profile-steps 0" ;;
  esac
  step pmc_${cfg}_a 90 timeout -s KILL 80 $P -o ${cfg}_a --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -- $B
  step pmc_${cfg}_b 90 timeout -s KILL 80 $P -o ${cfg}_b --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -- $B
  step pmc_${cfg}_c 90 timeout -s KILL 80 $P -o ${cfg}_c --pmc FETCH_SIZE -- $B
  step pmc_${cfg}_d 90 timeout -s KILL 80 $P -o ${cfg}_d --pmc WRITE_SIZE -- $B
done
