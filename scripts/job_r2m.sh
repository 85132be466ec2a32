#!/bin/bash
# fused5 MFMA core (BDX_F5_MFMA=1): correctness (fused5 tests with the MFMA
# instance forced on), interleaved A/B vs the VALU core, PMC MFMA count.
source scripts/gpu_steps.sh
BDX_F5_MFMA=1 step pytest_f5_mfma 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_runtime.py -q -rf --timeout 240 --timeout-method thread -k "fused5 or version5 or -5- or golden or segments"
B="python -u bench.py --steps 100 --warmup 5 --extras off --profile-steps 0"
for rep in 1 2; do
  for cfg in q6f32 q6; do
    BDX_F5_MFMA=0 step ab_${cfg}_valu_$rep 200 $B --config $cfg
    BDX_F5_MFMA=1 step ab_${cfg}_mfma_$rep 200 $B --config $cfg
  done
done
BDX_F5_MFMA=1 step pmc_mfma 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/pmc_mfma -o pmc -- python3 bench.py --config q6f32 --steps 3 --warmup 1 --extras off --profile-steps 0
BDX_F5_MFMA=0 step pmc_valu 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/pmc_valu -o pmc -- python3 bench.py --config q6f32 --steps 3 --warmup 1 --extras off --profile-steps 0
python - <<'PY'
import glob, json
for f in sorted(glob.glob('gpurun_out/ab_*.log')):
    for l in open(f):
        if l.startswith('{'):
            d = json.loads(l)
            print(f.split('/')[-1][:-4], round(d['value'], 2), d['config']['y_norm'])
PY
