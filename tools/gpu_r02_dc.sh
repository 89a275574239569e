#!/bin/bash
# deconv_px A/B, then the GPU suite (default path), then the parity files with omega_mfma
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python tools/variant_ab.py --planes 12 AARMVS_DECONV=old AARMVS_DECONV=px \
  AARMVS_OMEGA=mfma > gpurun_out/r02_dc_ab.log 2>&1; rc=$?
cut -c1-420 gpurun_out/r02_dc_ab.log; grep -o '"cost_max_diff_vs_first": [^,]*' gpurun_out/r02_dc_ab.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread \
  > gpurun_out/r02_dc_tests.log 2>&1; rc=$?
tail -4 gpurun_out/r02_dc_tests.log
[ $rc -eq 0 ] || exit $rc
AARMVS_OMEGA=mfma timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -q \
  --timeout 300 --timeout-method thread > gpurun_out/r02_mfma_tests.log 2>&1; rc=$?
tail -4 gpurun_out/r02_mfma_tests.log
exit 0
