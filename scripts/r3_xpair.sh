#!/bin/bash
# Round 3: paired lagged x update (fused5): GPU suite, then same-box
# interleaved A/B of BDX_XPAIR=1 (default) vs 0 on Q3 / Q6 / Q6-FP32.
source scripts/gpu_steps.sh
step xp_pytest 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
rm -f gpurun_out/xpair_summary.txt
for cfg in q3 q6 q6f32; do
  for rep in 1 2; do
    for v in 1 0; do
      step xp_${cfg}_${v}_$rep 300 env BDX_XPAIR=$v python -u bench.py --config $cfg --steps 100 --warmup 10 --companions off --extras off
      tail -1 gpurun_out/xp_${cfg}_${v}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['config']['phases_ms']; print('XP', '$cfg', 'xpair=$v', $rep, round(d['value'],3), round(d['ms_per_step_median'],4), round(p['op_interior'],4), round(p['update_rr'],4), d['config']['y_norm'])" | tee -a gpurun_out/xpair_summary.txt
    done
  done
done
