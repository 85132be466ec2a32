#!/bin/bash
# Kernel-trace + PMC profile of the flagship CG step (run on the GPU box).
# usage: scripts/prof_fused.sh <tag> [bench args...]
set -e
tag=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/$tag -o trace -- python3 bench.py "$@" > gpurun_out/prof/$tag.trace.log 2>&1
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/prof/$tag -o pmc1 -- python3 bench.py "$@" > gpurun_out/prof/$tag.pmc1.log 2>&1
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/prof/$tag -o pmc2 -- python3 bench.py "$@" > gpurun_out/prof/$tag.pmc2.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/prof/$tag -o pmc3 -- python3 bench.py "$@" > gpurun_out/prof/$tag.pmc3.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/$tag -o pmc4 -- python3 bench.py "$@" > gpurun_out/prof/$tag.pmc4.log 2>&1
