#!/bin/bash
# config 1's bimodality: four processes with HIP's default 4 hardware queues against four with
# GPU_MAX_HW_QUEUES=8, alternating, one box.
set -o pipefail
T=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3 4; do
  timeout -k 10 200 python bench.py --config plumbing_160x128_n3_d48 --steps 20 --warmup 3 --no-cpu --no-train --no-e2e --no-fusion --no-kernel-timing > gpurun_out/${T}_q4_$r.json 2> gpurun_out/${T}_q4_$r.err || exit 1
  GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python bench.py --config plumbing_160x128_n3_d48 --steps 20 --warmup 3 --no-cpu --no-train --no-e2e --no-fusion --no-kernel-timing > gpurun_out/${T}_q8_$r.json 2> gpurun_out/${T}_q8_$r.err || exit 1
done
for f in gpurun_out/${T}_q*_*.json; do python -c "
import json; d=json.load(open('$f')); print('$f'.split('/')[-1], round(d['value']/1e9,4), d['ms_per_step'])"; done
