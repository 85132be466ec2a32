#!/bin/bash
source scripts/gpu_steps.sh
P="rocprofv3 --output-format csv -d gpurun_out/pmcf2"
B="python3 bench.py --steps 3 --warmup 1 --config ${CFG:-q3} --kernel fused2"
step pmcf2_valu 240 $P -o valu --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SMEM SQ_INSTS_VALU -- $B
step pmcf2_wait 240 $P -o wait --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -- $B
step pmcf2_lds 240 $P -o lds --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_BRANCH GRBM_GUI_ACTIVE -- $B
