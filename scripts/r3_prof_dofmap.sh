set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3prof/dofmap -o run -- python3 bench.py --config q3 --kernel dofmap --geometry stored --steps 20 --warmup 3 --extras off --profile-steps 0 > gpurun_out/r3prof/dofmap.json 2> gpurun_out/r3prof/dofmap.err
find gpurun_out/r3prof/dofmap -name '*stats*' | head
