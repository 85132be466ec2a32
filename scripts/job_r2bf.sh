#!/bin/bash
# Same-box interleaved A/B of the segment cost model on the fused5 box
# configs: fractional rounds (new, default) vs whole rounds (wr).
CFGS="q3 q6f32 q6" VARIANTS="new wr" REPS=3 BENCH_EXTRA="--extras off" bash scripts/job_abvar.sh
