#!/bin/bash
# Round-6 step n: the regulariser as five units over 1-5 streams -- the bit-identity tests (eval
# and training record), then bench lines at configs 1, 2, 5 and the headline for 3 / 4 / 5 streams
# and the training step for 1 / 3 / 5.
set -o pipefail
mkdir -p gpurun_out
T=$1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bptt.py -x -q --timeout 300 --timeout-method thread \
  -k "multi_stream or streams_are_bit_identical or recorded or state" > gpurun_out/${T}_tests.log 2>&1 || { tail -20 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
run() {  # run NAME CONFIG REG extra...
  local n=$1 c=$2 r=$3; shift 3
  AARMVS_REG_STREAMS=$r timeout -k 10 300 python bench.py --config $c --no-cpu --no-train --no-e2e --no-fusion --no-kernel-timing "$@" > gpurun_out/${T}_$n.json 2> gpurun_out/${T}_$n.err || exit 1
}
for r in 1 3 4 5; do run c1_r$r plumbing_160x128_n3_d48 $r; done
for r in 3 4 5; do run c2_r$r dtu_eval_800x600_n5_d256 $r --steps 3; done
for r in 3 5; do run c5_r$r tnt_1920x1056_n11_d898 $r --steps 1 --warmup 1; done
for r in 3 4 5; do run h_r$r dtu_eval_1600x1184_n7_d512 $r --steps 2; done
for r in 1 3 5; do
  AARMVS_REG_STREAMS_REC=$r timeout -k 10 300 python -u bench.py --train --steps 6 --warmup 2 --no-cpu --no-kernel-timing \
    > gpurun_out/${T}_t_r$r.json 2> gpurun_out/${T}_t_r$r.err || exit 1
done
for f in gpurun_out/${T}_c*_r*.json gpurun_out/${T}_h_r*.json gpurun_out/${T}_t_r*.json; do python -c "
import json,sys; d=json.loads(open('$f').read().strip().split('\n')[-1]); print('$f'.split('/')[-1], d['value'], d['unit'], d['ms_per_step'], 'ms')"; done | tee gpurun_out/${T}_summary.txt
