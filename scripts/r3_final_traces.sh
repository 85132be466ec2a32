#!/bin/bash
# Kernel traces of the committed tree: Q3 headline and the dofmap data model.
source scripts/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step ft_q3 240 rocprofv3 --kernel-trace --stats -d gpurun_out/ft_q3 -o run -- python3 bench.py --config q3 --steps 30 --warmup 3 --companions off --extras off --profile-steps 0
step ft_dofmap 240 rocprofv3 --kernel-trace --stats -d gpurun_out/ft_dofmap -o run -- python3 bench.py --config q3 --kernel dofmap --geometry stored --steps 20 --warmup 3 --companions off --extras off --profile-steps 0
step ft_dofmap_q6 240 rocprofv3 --kernel-trace --stats -d gpurun_out/ft_dofmap_q6 -o run -- python3 bench.py --config q6 --kernel dofmap --geometry stored --steps 10 --warmup 2 --companions off --extras off --profile-steps 0
