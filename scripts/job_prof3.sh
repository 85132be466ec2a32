#!/bin/bash
source scripts/gpu_steps.sh
for c in q3 q6; do
  step trace_$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof3_$c -o trace -- python3 bench.py --steps 20 --warmup 2 --config $c
  B="python3 bench.py --steps 3 --warmup 1 --config $c"
  P="rocprofv3 --output-format csv -d gpurun_out/prof3_$c"
  step pmcA_$c 240 $P -o pmcA --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -- $B
  step pmcB_$c 240 $P -o pmcB --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -- $B
  step pmcC_$c 240 $P -o pmcC --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SMEM SQ_LDS_IDX_ACTIVE -- $B
done
