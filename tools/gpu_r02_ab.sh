#!/bin/bash
# Round-2: GPU tests (default = omega_mfma), then omega variant A/B timing, then a bench line.
set -o pipefail
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread \
  > gpurun_out/r02_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r02_tests.log | tail -60
if fatal $rc; then echo "tests died rc=$rc"; tail -30 gpurun_out/r02_tests.log; exit 1; fi
timeout -k 10 300 python tools/variant_ab.py --planes 24 AARMVS_OMEGA=valu AARMVS_OMEGA=mfma \
  > gpurun_out/r02_ab.log 2>&1 || { echo "AB FAILED"; tail -30 gpurun_out/r02_ab.log; exit 1; }
cat gpurun_out/r02_ab.log
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/r02_bench.log 2>&1 || { echo BENCH FAILED; tail -30 gpurun_out/r02_bench.log; exit 1; }
tail -c 4000 gpurun_out/r02_bench.log
exit $rc
