#!/bin/bash
# Round-6 step r: one library stream pool shared by the sweep and the backward (four streams per
# process), the small-frame schedule with the aux stream as a unit stream -- tests, bench lines,
# and a kernel trace of the training step (which hardware queue each stream ran on)
set -o pipefail
mkdir -p gpurun_out
T=$1
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bptt.py tests/test_gpu_training.py -x -q --timeout 400 --timeout-method thread \
  > gpurun_out/${T}_tests.log 2>&1 || { tail -20 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
run() {  # run NAME CONFIG SMALL_PX extra...
  local n=$1 c=$2 px=$3; shift 3
  AARMVS_SMALL_PX=$px timeout -k 10 300 python bench.py --config $c --no-cpu --no-train --no-e2e --no-fusion --no-kernel-timing "$@" > gpurun_out/${T}_$n.json 2> gpurun_out/${T}_$n.err || exit 1
}
run c1_def plumbing_160x128_n3_d48 65536
run c1_big plumbing_160x128_n3_d48 0
run c2_def dtu_eval_800x600_n5_d256 65536 --steps 3
run h_def dtu_eval_1600x1184_n7_d512 65536 --steps 2
timeout -k 10 300 python -u bench.py --train --steps 6 --warmup 2 --no-cpu --no-kernel-timing > gpurun_out/${T}_t.json 2> gpurun_out/${T}_t.err || exit 1
for f in gpurun_out/${T}_*.json; do python -c "
import json,sys; d=json.loads(open('$f').read().strip().split('\n')[-1]); print('$f'.split('/')[-1], d['value'], d['unit'], d['ms_per_step'], 'ms')"; done | tee gpurun_out/${T}_summary.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${T}_trt -o run -- \
  python3 $R/bench.py --train --steps 2 --warmup 1 --no-cpu --no-kernel-timing > $R/gpurun_out/${T}_trt.log 2>&1 || exit 1
f=$(find $R/gpurun_out/${T}_trt -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_streams.py $f 230 gate_bwd > $R/gpurun_out/${T}_train_streams.txt && head -12 $R/gpurun_out/${T}_train_streams.txt
