#!/bin/bash
# Round-6 step q: the small-frame schedule (cost stage on the caller's stream, units over four
# streams) -- bit-identity tests, then config 1 by default, and configs 2 / headline with the
# small-frame schedule forced (AARMVS_SMALL_PX) against their default
set -o pipefail
mkdir -p gpurun_out
T=$1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bptt.py -x -q --timeout 300 --timeout-method thread \
  -k "multi_stream or streams_are_bit_identical" > gpurun_out/${T}_tests.log 2>&1 || { tail -20 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
run() {  # run NAME CONFIG SMALL_PX extra...
  local n=$1 c=$2 px=$3; shift 3
  AARMVS_SMALL_PX=$px timeout -k 10 300 python bench.py --config $c --no-cpu --no-train --no-e2e --no-fusion --no-kernel-timing "$@" > gpurun_out/${T}_$n.json 2> gpurun_out/${T}_$n.err || exit 1
}
run c1_def plumbing_160x128_n3_d48 65536
run c1_big plumbing_160x128_n3_d48 0
run c2_def dtu_eval_800x600_n5_d256 65536 --steps 3
run c2_small dtu_eval_800x600_n5_d256 100000000 --steps 3
run h_def dtu_eval_1600x1184_n7_d512 65536 --steps 2
run h_small dtu_eval_1600x1184_n7_d512 100000000 --steps 2
run c1_def2 plumbing_160x128_n3_d48 65536
for f in gpurun_out/${T}_*.json; do python -c "
import json,sys; d=json.loads(open('$f').read().strip().split('\n')[-1]); print('$f'.split('/')[-1], round(d['value']/1e9, 4), 'G', d['ms_per_step'], 'ms')"; done | tee gpurun_out/${T}_summary.txt
