#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/debug_omega.py 1184 1600 7 > gpurun_out/r02_dbg3.log 2>&1; rc=$?
grep -v Warn gpurun_out/r02_dbg3.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/variant_ab.py --planes 16 AARMVS_OMEGA=valu AARMVS_OMEGA=mfma \
  AARMVS_OMEGA=mfma,AB_OVERLAP=0 > gpurun_out/r02_ab2.log 2>&1; rc=$?
cut -c1-600 gpurun_out/r02_ab2.log; grep -o '"cost_max_diff_vs_first": [^,]*' gpurun_out/r02_ab2.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 400 --timeout-method thread > gpurun_out/r02_tests2.log 2>&1; rc=$?
tail -5 gpurun_out/r02_tests2.log
exit $rc
