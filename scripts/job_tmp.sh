source scripts/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export BDX_PROBE_OUT=gpurun_out/r4_overlap_probe.jsonl
step r4a_pytest 600 python -u -m pytest tests/test_gpu_overlap_probe.py tests/test_gpu_rccl.py tests/test_gpu_runtime.py -x -v --timeout 120 --timeout-method thread
step r4a_driver 400 python -u bench.py --gpus 1 --steps 20 --warmup 5
