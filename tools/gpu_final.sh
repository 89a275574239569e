#!/bin/bash
# Round measurement: the GPU test suite, smoke(), the default bench line (headline + CPU
# baseline + fusion + e2e + config-4 training step) and a rocprofv3 kernel-trace/stats run of
# the headline sweep.  Each step has its own time limit; anything but pass/fail ends the run.
# usage: bash tools/gpu_final.sh TAG
set -u
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step NAME SECONDS cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -2 "gpurun_out/${TAG}_$name.log" | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step tests 540 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 420 python -u bench.py
step prof 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$TAG -o ks -- \
  python3 bench.py --no-cpu --no-fusion --no-e2e --no-train --steps 2
for f in $(find /tmp/prof_$TAG -name "ks_kernel_stats.csv"); do cp "$f" gpurun_out/${TAG}_kernel_stats.csv; done
