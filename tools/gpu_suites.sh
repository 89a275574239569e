#!/bin/bash
# GPU suite on the default path, then the parity files with the VALU omega_conv selected
# (the A/B of the two omega variants)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/r02_tests3.log 2>&1; rc=$?
tail -4 gpurun_out/r02_tests3.log
[ $rc -eq 0 ] || exit $rc
AARMVS_OMEGA=valu timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_models.py -m gpu -q \
  --timeout 300 --timeout-method thread > gpurun_out/r02_mfma_tests.log 2>&1; rc=$?
tail -6 gpurun_out/r02_mfma_tests.log
exit $rc
