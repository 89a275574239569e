#!/bin/bash
# Kernel traces (rocprofv3 --kernel-trace, CSV copied to gpurun_out/): the headline sweep over
# its first 64 planes (two streams, no per-launch events: the overlap of the two streams) and
# the config-4 backward probe (tools/cbf_probe.py).  usage: bash tools/gpu_trace.sh TAG
set -u
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/tr_$TAG -o fwd -- \
  python3 bench.py --no-cpu --no-fusion --no-e2e --no-train --no-kernel-timing --planes 64 --steps 2 \
  > gpurun_out/${TAG}_fwd.log 2>&1 || exit $?
for f in $(find /tmp/tr_$TAG -name "fwd_kernel_trace.csv"); do cp "$f" gpurun_out/${TAG}_fwd_trace.csv; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/tb_$TAG -o bwd -- \
  python3 tools/cbf_probe.py > gpurun_out/${TAG}_bwd.log 2>&1 || exit $?
for f in $(find /tmp/tb_$TAG -name "bwd_kernel_trace.csv"); do python3 tools/trace_summary.py "$f" gpurun_out/${TAG}_bwd_grid.csv; done
