#!/bin/bash
# GPU check after a change: the full GPU test suite, then a short headline bench line
# (no CPU / fusion / e2e legs).  usage: bash tools/gpu_check.sh <tag> [extra bench args]
set -o pipefail
tag=${1:-chk}; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${tag}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-fusion --no-e2e "$@" \
  > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err; rc=$?
cut -c1-600 gpurun_out/${tag}_bench.json
exit $rc
