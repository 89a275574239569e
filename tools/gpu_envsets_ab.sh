#!/bin/bash
# Headline bench and sweep digest under several environment sets, twice in turn:
# bash tools/gpu_envsets_ab.sh TAG "A=1 B=0" "A=0 B=0" ...  -> gpurun_out/TAG_<i>_<r>.json
set -o pipefail
mkdir -p gpurun_out
tag=$1; shift
for r in 1 2; do
  i=0
  for set in "$@"; do
    env $set timeout -k 10 300 python bench.py --steps 2 --no-cpu --no-train --no-e2e --no-fusion > gpurun_out/${tag}_${i}_$r.json 2>/dev/null || exit 1
    i=$((i+1))
  done
done
for set in "$@"; do
  env $set timeout -k 10 200 python tools/sweep_digest.py >> gpurun_out/${tag}_digest.txt 2>&1 || exit 1
done
