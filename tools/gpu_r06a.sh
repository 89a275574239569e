#!/bin/bash
# Round-6 baseline on the round-5 tree: the headline line (kernel timing, no CPU leg) and the
# other configs' lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --no-cpu --no-train --no-e2e --no-fusion > gpurun_out/$1_head.json 2> gpurun_out/$1_head.err && \
bash tools/gpu_configs.sh $1
