#!/bin/bash
source scripts/gpu_steps.sh
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
P="rocprofv3 --output-format csv -d gpurun_out/pmc2"
step pmc_valu 240 $P -o valu --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_SMEM -- python3 bench.py --steps 3 --warmup 1 --config q3
step pmc_misc 240 $P -o misc --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_BRANCH SQ_INSTS_SENDMSG SQ_WAVE_CYCLES -- python3 bench.py --steps 3 --warmup 1 --config q3
step bench_q3_stored 300 python -u bench.py --steps 10 --warmup 2 --config q3 --geometry stored
step bench_q3_v1 300 python -u bench.py --steps 5 --warmup 1 --config q3 --kernel v1
