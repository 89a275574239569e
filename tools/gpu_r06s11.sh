#!/bin/bash
# omega_conv items per block (AARMVS_OMEGA_IPB) on the final kernel: headline bench lines
# default / 8 / 2 / default / 8, one box.
set -o pipefail
T=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for ipb in def 8 2 def 8; do
  i=$((i+1))
  if [ $ipb = def ]; then unset AARMVS_OMEGA_IPB; else export AARMVS_OMEGA_IPB=$ipb; fi
  timeout -k 10 300 python bench.py --steps 2 --no-cpu --no-train --no-e2e --no-fusion > gpurun_out/${T}_${i}_ipb$ipb.json 2> gpurun_out/${T}_${i}.err || exit 1
done
python tools/ab_summary.py gpurun_out/${T}_*_ipb*.json
