#!/bin/bash
# Headline bench A/B/A/B of an environment switch: bash tools/gpu_env_ab.sh TAG VAR VAL_A VAL_B
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in $3 $4; do
    env $2=$v timeout -k 10 300 python bench.py --steps 2 --no-cpu --no-train --no-e2e --no-fusion > gpurun_out/$1_${v}_$r.json 2> gpurun_out/$1_${v}_$r.err || exit 1
  done
done
