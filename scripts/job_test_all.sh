#!/bin/bash
source scripts/gpu_steps.sh
step micro 120 benchmark_dolfinx_amd/csrc/micro/f64_pipes.bin
step pytest_gpu 1200 python -m pytest tests -m gpu -x -q
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 600 python -u bench.py
