#!/bin/bash
# Round-6 step l: the float64 backward tests with the uniform bound and the new omega-bias test
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_bptt.py -x -v -s --timeout 400 --timeout-method thread -k "float64 or systematic" > gpurun_out/$1_bptt.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|seed|bias" gpurun_out/$1_bptt.log | head -30
exit $rc
