#!/bin/bash
# deformable sampling timing A/B (in-tree vs tools/ab/lib_$1.so), then the deform GPU tests
set -o pipefail
for i in 1 2; do
  timeout -k 10 120 python tools/deform_time.py || exit 1
  AARMVS_LIB=$PWD/tools/ab/lib_$1.so timeout -k 10 120 python tools/deform_time.py || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_deform.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3
