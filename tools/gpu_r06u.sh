#!/bin/bash
# Round-6 step u: the stream bit-identity tests with their large-frame cases
set -o pipefail
mkdir -p gpurun_out
T=$1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bptt.py -x -q --timeout 400 --timeout-method thread \
  -k "multi_stream or streams_are_bit_identical" > gpurun_out/${T}_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${T}_tests.log
exit $rc
