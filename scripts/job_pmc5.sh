#!/bin/bash
# fused5 PMC passes (Q6 FP64): wave occupancy, stall reasons, instruction mix, HBM bytes.
source scripts/gpu_steps.sh
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
P="rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc5"
B="python3 bench.py --steps 3 --warmup 1 --config ${CFG:-q6} --kernel fused5"
step pmc5_a 90 timeout -s KILL 80 $P -o a --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -- $B
step pmc5_b 90 timeout -s KILL 80 $P -o b --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -- $B
step pmc5_c 90 timeout -s KILL 80 $P -o c --pmc FETCH_SIZE -- $B
step pmc5_d 90 timeout -s KILL 80 $P -o d --pmc WRITE_SIZE -- $B
step pmc5_e 90 timeout -s KILL 80 $P -o e --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_EXP SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VMEM SQ_INSTS_WAVE32 GRBM_GUI_ACTIVE -- $B
