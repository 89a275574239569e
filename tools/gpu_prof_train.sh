#!/bin/bash
# Training-step kernel profile: rocprofv3 kernel trace + stats of tools/train_step.py; the raw
# output stays in /tmp, the stats CSVs are copied into gpurun_out/.
# usage: bash tools/gpu_prof_train.sh TAG [train_step args...]
set -u
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$TAG -o run \
  -- python3 ${PROF_SCRIPT:-tools/train_step.py} "$@" > gpurun_out/${TAG}_prof.log 2>&1
rc=$?
grep -v "^W2026" gpurun_out/${TAG}_prof.log | tail -3
for f in $(find /tmp/prof_$TAG -name "*kernel_stats.csv"); do cp "$f" gpurun_out/${TAG}_kernel_stats.csv; done
for f in $(find /tmp/prof_$TAG -name "*kernel_trace.csv"); do
  python3 tools/trace_summary.py "$f" gpurun_out/${TAG}_kernel_grid.csv
done
exit $rc
