#!/bin/bash
# Round-6 step o: config 1 (160x128) with the regulariser's units over up to 4 streams when the
# cost stage shares the caller's stream (--no-overlap: caller + 3 library streams = 4 hardware
# queues), against the default (cost stage on the aux stream, 3 unit streams); and 5 unit
# streams with 8 hardware queues (is r06n's 4/5-stream slowdown queue sharing?)
set -o pipefail
mkdir -p gpurun_out
T=$1
run() {  # run NAME REG MAP extra...
  local n=$1 r=$2 m=$3; shift 3
  AARMVS_REG_STREAMS=$r AARMVS_REG_MAP=$m timeout -k 10 200 python bench.py --config plumbing_160x128_n3_d48 --no-cpu --no-train --no-e2e --no-fusion --no-kernel-timing "$@" > gpurun_out/${T}_$n.json 2> gpurun_out/${T}_$n.err || exit 1
}
run ov_r3 3 ""
run no_r1 1 "" --no-overlap
run no_r3 3 "" --no-overlap
run no_r4 4 "" --no-overlap
run no_00123 4 00123 --no-overlap
run no_01223 4 01223 --no-overlap
run no_01233 4 01233 --no-overlap
run no_00012 3 00012 --no-overlap
run ov_r2 2 ""
GPU_MAX_HW_QUEUES=8 run ov_r5_q8 5 ""
GPU_MAX_HW_QUEUES=8 run ov_r3_q8 3 ""
for f in gpurun_out/${T}_*.json; do python -c "
import json,sys; d=json.loads(open('$f').read().strip().split('\n')[-1]); print('$f'.split('/')[-1], round(d['value']/1e9, 4), 'G', d['ms_per_step'], 'ms')"; done | tee gpurun_out/${T}_summary.txt
