#!/bin/bash
# a quick subset of the GPU tests (args: pytest selectors; default: the configs + eval files)
set -o pipefail
mkdir -p gpurun_out
sel=${@:-tests/test_gpu_configs.py tests/test_gpu_eval.py}
timeout -k 10 400 python -u -m pytest $sel -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/quick_tests.log 2>&1; rc=$?
tail -8 gpurun_out/quick_tests.log
exit $rc
