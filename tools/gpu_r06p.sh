#!/bin/bash
# Round-6 step p: kernel traces of config 1 (160x128, D=48) with the regulariser's units on 3 and
# on 5 streams: which hardware queue each stream's kernels ran on, busy vs idle, kernel times
set -o pipefail
T=$1
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for r in 3 5; do
  AARMVS_REG_STREAMS=$r timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${T}_tr$r -o run -- \
    python3 $R/bench.py --config plumbing_160x128_n3_d48 --steps 2 --warmup 1 --no-cpu --no-train --no-e2e --no-fusion \
    --no-kernel-timing > $R/gpurun_out/${T}_tr$r.log 2>&1 || exit 1
  f=$(ls $R/gpurun_out/${T}_tr$r/*kernel_trace.csv 2>/dev/null || find $R/gpurun_out/${T}_tr$r -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/trace_streams.py $f 3.5 > $R/gpurun_out/${T}_streams_r$r.txt || exit 1
  head -12 $R/gpurun_out/${T}_streams_r$r.txt
done
