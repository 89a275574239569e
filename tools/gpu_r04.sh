#!/bin/bash
# Round-4 GPU session: named tests first, then (unless SUITE=0) the whole GPU suite and smoke,
# then bench.py with the given arguments (none: no bench).  Each step has its own time limit;
# a crash, abort or timeout ends the session (rc 0 = pass, 1 = test failures, else stop).
# usage: bash tools/gpu_r04.sh TAG "pytest selection" [bench args...]
set -u
TAG=$1; SEL=$2; shift 2
mkdir -p gpurun_out
step() {  # step <name> <seconds> cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a gpurun_out/${TAG}_session.log
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/${TAG}_session.log
  tail -4 "gpurun_out/${TAG}_$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
if [ -n "$SEL" ]; then
  step sel 900 python -u -m pytest $SEL -v -s --timeout 300 --timeout-method thread
fi
if [ "${SUITE:-1}" != "0" ]; then
  step gpu 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
  step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
fi
if [ $# -gt 0 ]; then
  step bench 900 python -u bench.py "$@"
fi
