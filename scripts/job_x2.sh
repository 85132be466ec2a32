#!/bin/bash
# Two-step lagged x update (fused4/5): GPU suite + same-box A/B vs HEAD.
source scripts/gpu_steps.sh

CFGS="q3 q6 q6f32" VARIANTS="x1 new" REPS=2 bash scripts/job_abvar.sh
