#!/bin/bash
# Headline bench: tools/ab/lib_$1.so vs the in-tree library under env VAR=VAL, A/B/A/B,
# plus a digest of each: bash tools/gpu_ab3.sh LIBTAG VAR VAL
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  AARMVS_LIB=$PWD/tools/ab/lib_$1.so timeout -k 10 300 python bench.py --steps 2 --no-cpu --no-train --no-e2e --no-fusion > gpurun_out/ab3_$1_$r.json 2>/dev/null || exit 1
  env $2=$3 timeout -k 10 300 python bench.py --steps 2 --no-cpu --no-train --no-e2e --no-fusion > gpurun_out/ab3_new_$r.json 2>/dev/null || exit 1
done
AARMVS_LIB=$PWD/tools/ab/lib_$1.so timeout -k 10 200 python tools/sweep_digest.py >> gpurun_out/ab3_digest.txt 2>&1 || exit 1
env $2=$3 timeout -k 10 200 python tools/sweep_digest.py >> gpurun_out/ab3_digest.txt 2>&1
