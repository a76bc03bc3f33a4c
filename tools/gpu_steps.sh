#!/bin/bash
# GPU-box helper: run steps in order, each under its own time limit; a pytest failure (rc 1) lets the
# next step run, anything else (fault, abort, timeout, crash) ends the call there.
# usage: source tools/gpu_steps.sh; step <seconds> <log> <cmd...>
mkdir -p gpurun_out
step() {
  local secs=$1 log=$2
  shift 2
  echo "[step] $* (limit ${secs}s) -> $log"
  timeout -k 10 "$secs" "$@" > "$log" 2>&1
  local rc=$?
  echo "[step] rc=$rc"
  tail -3 "$log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "[step] stopping: rc=$rc"
    exit $rc
  fi
}
