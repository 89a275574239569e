#!/bin/bash
# Round-6 step f: the two-stream regulariser (AARMVS_REG_STREAMS) -- its bit-identity tests, then
# bench lines with it off and on at configs 1 and 2 and the headline.
set -o pipefail
mkdir -p gpurun_out
T=$1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "two_stream" > gpurun_out/${T}_tests.log 2>&1 || { tail -20 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
run() {  # run NAME CONFIG REG extra...
  local n=$1 c=$2 r=$3; shift 3
  AARMVS_REG_STREAMS=$r timeout -k 10 300 python bench.py --config $c --no-cpu --no-train --no-e2e --no-fusion "$@" > gpurun_out/${T}_$n.json 2> gpurun_out/${T}_$n.err || exit 1
}
run c1_r0 plumbing_160x128_n3_d48 1
run c1_r1 plumbing_160x128_n3_d48 1
run c2_r0 dtu_eval_800x600_n5_d256 0 --steps 3
run c2_r1 dtu_eval_800x600_n5_d256 1 --steps 3
run h_r0 dtu_eval_1600x1184_n7_d512 0 --steps 2
run h_r1 dtu_eval_1600x1184_n7_d512 1 --steps 2
python tools/ab_summary.py gpurun_out/${T}_c1_r0.json gpurun_out/${T}_c1_r1.json gpurun_out/${T}_c2_r0.json gpurun_out/${T}_c2_r1.json gpurun_out/${T}_h_r0.json gpurun_out/${T}_h_r1.json
