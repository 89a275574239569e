#!/bin/bash
# kernel-variant A/B at the headline geometry (tools/variant_ab.py); args: variants
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python tools/variant_ab.py --planes 12 "$@" > gpurun_out/ab.log 2>&1; rc=$?
cut -c1-330 gpurun_out/ab.log; grep -o '"cost_max_diff_vs_first": [^,]*' gpurun_out/ab.log
exit $rc
