#!/bin/bash
# Backward A/B over one 16-plane group (tools/cbf_probe.py: time + output digest), in-tree
# library vs tools/ab/lib_$1.so, twice, under rocprofv3 kernel statistics for the second pair
set -o pipefail
for i in 1 2; do
  timeout -k 10 120 python tools/cbf_probe.py || exit 1
  AARMVS_LIB=$PWD/tools/ab/lib_$1.so timeout -k 10 120 python tools/cbf_probe.py || exit 1
done
