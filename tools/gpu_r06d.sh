#!/bin/bash
# Round-6 step d: digest of the in-tree library (expected equal to round 5's), the HIP-graph
# probe at configs 1 and 2, and the omega/cost_x ceiling counters of the in-tree library.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python tools/sweep_digest.py > gpurun_out/$1_digest.txt 2>&1 || exit 1
cat gpurun_out/$1_digest.txt
timeout -k 10 120 python tools/graph_probe.py > gpurun_out/$1_graph1.txt 2>&1 || exit 1
cat gpurun_out/$1_graph1.txt | tail -1
timeout -k 10 200 python tools/graph_probe.py 5 600 800 256 > gpurun_out/$1_graph2.txt 2>&1 || exit 1
cat gpurun_out/$1_graph2.txt | tail -1
CEIL_DIR=gpurun_out/$1_ceil bash tools/gpu_ceiling.sh || exit 1
python tools/ceiling_summary.py gpurun_out/$1_ceil > gpurun_out/$1_ceil_summary.txt 2>&1
tail -30 gpurun_out/$1_ceil_summary.txt
