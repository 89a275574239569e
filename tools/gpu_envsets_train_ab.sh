#!/bin/bash
# Headline bench with the training section under several environment sets, twice in turn:
# bash tools/gpu_envsets_train_ab.sh TAG "A=1" "A=0" ...  -> gpurun_out/TAG_<i>_<r>.json
set -o pipefail
mkdir -p gpurun_out
tag=$1; shift
for r in 1 2; do
  i=0
  for set in "$@"; do
    env $set timeout -k 10 400 python bench.py --steps 2 --no-cpu --no-e2e --no-fusion > gpurun_out/${tag}_${i}_$r.json 2>/dev/null || exit 1
    i=$((i+1))
  done
done
