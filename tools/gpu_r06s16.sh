#!/bin/bash
# config 1 (160x128, N=3, D=48, 20 timed steps): the r06f tree's library (tools/ab/lib_r06f.so) against
# the in-tree one, A/B three times on one box.
set -o pipefail
T=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
  AARMVS_LIB=$PWD/tools/ab/lib_r06f.so timeout -k 10 200 python bench.py --config plumbing_160x128_n3_d48 --steps 20 --warmup 3 --no-cpu --no-train --no-e2e --no-fusion --no-kernel-timing > gpurun_out/${T}_A_$r.json 2> gpurun_out/${T}_A_$r.err || exit 1
  timeout -k 10 200 python bench.py --config plumbing_160x128_n3_d48 --steps 20 --warmup 3 --no-cpu --no-train --no-e2e --no-fusion --no-kernel-timing > gpurun_out/${T}_B_$r.json 2> gpurun_out/${T}_B_$r.err || exit 1
done
for f in gpurun_out/${T}_[AB]_*.json; do python -c "
import json; d=json.load(open('$f')); print('$f'.split('/')[-1], round(d['value']/1e9,4), d['ms_per_step'])"; done
