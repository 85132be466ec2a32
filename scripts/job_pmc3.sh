#!/bin/bash
# fused3 PMC passes (Q3 / Q6): instruction mix, LDS waits and conflicts, HBM bytes.
source scripts/gpu_steps.sh
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
P="rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc3"
for cfg in q3 q6; do
step pmc_${cfg}_a 90 timeout -s KILL 80 $P -o ${cfg}_a --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS -- python3 bench.py --steps 3 --warmup 1 --config $cfg
step pmc_${cfg}_b 90 timeout -s KILL 80 $P -o ${cfg}_b --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -- python3 bench.py --steps 3 --warmup 1 --config $cfg
step pmc_${cfg}_c 90 timeout -s KILL 80 $P -o ${cfg}_c --pmc FETCH_SIZE WRITE_SIZE -- python3 bench.py --steps 3 --warmup 1 --config $cfg
done
