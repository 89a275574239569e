#!/bin/bash
# Round-4 rocprofv3 kernel statistics (--kernel-trace --stats, CSV): the config-4 training step
# (tools/train_step.py, one timed step after a warm-up) and the headline sweep (bench.py, two
# steps, no side legs); stats copied to gpurun_out/TAG_{train,head}_kernel_stats.csv.
# usage: bash tools/gpu_prof_r04.sh TAG
set -u
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pt_$TAG -o train -- \
  python3 tools/train_step.py --steps 1 > gpurun_out/${TAG}_train.log 2>&1 || exit $?
for f in $(find /tmp/pt_$TAG -name "train_kernel_stats.csv"); do cp "$f" gpurun_out/${TAG}_train_kernel_stats.csv; done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ph_$TAG -o head -- \
  python3 bench.py --no-cpu --no-fusion --no-e2e --no-train --steps 2 --warmup 1 > gpurun_out/${TAG}_head.log 2>&1 || exit $?
for f in $(find /tmp/ph_$TAG -name "head_kernel_stats.csv"); do cp "$f" gpurun_out/${TAG}_head_kernel_stats.csv; done
