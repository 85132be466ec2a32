#!/bin/bash
source scripts/gpu_steps.sh
step pytest_fused 900 python -m pytest tests/test_gpu_fused.py tests/test_gpu_distributed_emulated.py -x -q
for c in q3 q6 q6f32; do
  step bench_$c 300 python -u bench.py --steps 30 --warmup 3 --config $c
done
P="rocprofv3 --output-format csv -d gpurun_out/prof3b"
step pmc_q3 240 $P -o q3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -- python3 bench.py --steps 3 --warmup 1 --config q3
step pmc_q6 240 $P -o q6 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -- python3 bench.py --steps 3 --warmup 1 --config q6
grep -h '^{' gpurun_out/bench_*.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['config']['model'][:3], d['dtype'], d['config']['kernel'], round(d['value'], 3), round(d['ms_per_step'], 3), d['config']['y_norm'])
" || true
