#!/bin/bash
# fused4: full GPU numerics, kernel table, PMC passes (one counter block set per run).
source scripts/gpu_steps.sh
step pytest_f4 600 python -u -m pytest tests/test_gpu_fused.py -q --timeout 120 --timeout-method thread -k "fused4 or 4-True or -4-"
step prof_f4 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_f4 -o f4 -- python3 bench.py --steps 20 --warmup 2 --kernel fused4
P="rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc4"
B="python3 bench.py --steps 3 --warmup 1 --kernel fused4"
step pmc4_a 90 timeout -s KILL 80 $P -o a --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES -- $B
step pmc4_b 90 timeout -s KILL 80 $P -o b --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE -- $B
step pmc4_c 90 timeout -s KILL 80 $P -o c --pmc FETCH_SIZE -- $B
step pmc4_d 90 timeout -s KILL 80 $P -o d --pmc WRITE_SIZE -- $B
step pmc4_e 90 timeout -s KILL 80 $P -o e --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_VALU2 SQ_INSTS_SMEM SQ_INSTS_VMEM_RD -- $B
