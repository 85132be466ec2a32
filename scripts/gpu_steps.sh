#!/bin/bash
# Helper sourced by GPU-box job scripts: run named steps with their own time
# limit, log to gpurun_out/<name>.log, and stop the whole job after a fatal
# status (fault/abort/segv/timeout).  Plain test failures (exit 1) continue.
#   source scripts/gpu_steps.sh; step NAME SECONDS cmd args...
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {
  local name=$1 secs=$2
  shift 2
  echo "[step] $name: $*" | tee -a gpurun_out/steps.log
  local t0=$(date +%s)
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[step] $name rc=$rc ($(( $(date +%s) - t0 ))s)" | tee -a gpurun_out/steps.log
  tail -n 5 "gpurun_out/$name.log"
  case $rc in
    0|1|5) return 0 ;;
    *) echo "[step] fatal status $rc in $name: stopping" | tee -a gpurun_out/steps.log; exit $rc ;;
  esac
}
