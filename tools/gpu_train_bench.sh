#!/bin/bash
# training-step leg of bench.py alone (headline sweep skipped down to 2 planes)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --train --no-cpu --no-fusion --no-e2e --no-kernel-timing --planes 2 --steps 1 \
  > gpurun_out/train_bench.log 2>&1; rc=$?
tail -3 gpurun_out/train_bench.log | cut -c1-2000
exit $rc
