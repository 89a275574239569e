#!/bin/bash
# Round-6 step x: the sweep under HIP-graph capture (one stream while capturing) -- the parity
# test, then the probe's eager / graph timing at config 1
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "graph_capture or multi_stream" \
  > gpurun_out/$1_tests.log 2>&1 || { tail -20 gpurun_out/$1_tests.log; exit 1; }
tail -2 gpurun_out/$1_tests.log
timeout -k 10 200 python -u tools/graph_probe.py > gpurun_out/$1_graph.txt 2>&1 || { tail -5 gpurun_out/$1_graph.txt; exit 1; }
tail -1 gpurun_out/$1_graph.txt
