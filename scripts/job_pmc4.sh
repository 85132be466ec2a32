#!/bin/bash
# fused4 (Q3) and fused5 (Q6) PMC passes on the committed tree: MFMA / VALU
# activity, LDS bank conflicts, HBM bytes, wave occupancy.  One counter group
# per run (rocprofv3 does not split passes).
source scripts/gpu_steps.sh
P="rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc"
for cfg in q3 q6; do
  B="python3 bench.py --steps 3 --warmup 1 --config $cfg"
  step pmc_${cfg}_a 90 timeout -s KILL 80 $P -o ${cfg}_a --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -- $B
  step pmc_${cfg}_b 90 timeout -s KILL 80 $P -o ${cfg}_b --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -- $B
  step pmc_${cfg}_c 90 timeout -s KILL 80 $P -o ${cfg}_c --pmc FETCH_SIZE -- $B
  step pmc_${cfg}_d 90 timeout -s KILL 80 $P -o ${cfg}_d --pmc WRITE_SIZE -- $B
done
