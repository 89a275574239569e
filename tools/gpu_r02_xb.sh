#!/bin/bash
# cost_x variants A/B (gather / LDS box at 4 and 6 waves per SIMD) + omega_mfma check;
# fusion mask mismatch counts
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/fusion_mismatch.py > gpurun_out/r02_fusion_mm.log 2>&1; rc=$?
cat gpurun_out/r02_fusion_mm.log | grep -v Warn
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python tools/variant_ab.py --planes 12 AARMVS_COSTX=gather AARMVS_COSTX=box \
  AARMVS_COSTX=box6 AARMVS_OMEGA=mfma > gpurun_out/r02_xb_ab.log 2>&1; rc=$?
cut -c1-400 gpurun_out/r02_xb_ab.log; grep -o '"cost_max_diff_vs_first": [^,]*' gpurun_out/r02_xb_ab.log
exit $rc
