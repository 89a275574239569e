#!/bin/bash
# GPU-box session: parity tests, smoke, bench.  Stops at the first crash/timeout.
# usage: bash tools/gpu_round.sh [bench args...]
set -u
mkdir -p gpurun_out
run() {  # run <name> <timeout> cmd...  ; exit code 0/1 ok (1 = test failure), others stop
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a gpurun_out/session.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/session.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
