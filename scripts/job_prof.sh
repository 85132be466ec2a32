#!/bin/bash
# PMC profile of the flagship CG step + FP64 pipe microbenchmark.
source scripts/gpu_steps.sh
step micro_f64 120 benchmark_dolfinx_amd/csrc/micro/f64_pipes.bin
step prof_pmc 900 bash scripts/prof_fused.sh ${TAG:-q3} --steps 5 --warmup 1 --config ${CFG:-q3}
step prof_summary 60 python scripts/summarize_prof.py gpurun_out/prof/${TAG:-q3}
