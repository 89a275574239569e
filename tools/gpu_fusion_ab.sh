#!/bin/bash
# fusion-core timing A/B (in-tree vs tools/ab/lib_$1.so), then the fusion GPU tests
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 120 python tools/fusion_time.py 30 || exit 1
  AARMVS_LIB=$PWD/tools/ab/lib_$1.so timeout -k 10 120 python tools/fusion_time.py 30 || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_fusion.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3
