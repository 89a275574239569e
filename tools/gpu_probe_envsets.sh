#!/bin/bash
# Backward probe (tools/cbf_probe.py: time + digest over one 16-plane group) under several
# environment sets, twice in turn: bash tools/gpu_probe_envsets.sh "A=1" "A=0" ...
set -o pipefail
for r in 1 2; do
  for set in "$@"; do
    echo -n "[$set] "
    env $set timeout -k 10 120 python tools/cbf_probe.py || exit 1
  done
done
