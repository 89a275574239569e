#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/xsplit_check.py && \
AARMVS_XSPLIT=1 timeout -k 10 300 python bench.py --steps 2 --no-cpu --no-train --no-e2e --no-fusion > gpurun_out/$1_x1.json 2> gpurun_out/$1_x1.err && \
AARMVS_XSPLIT=0 timeout -k 10 300 python bench.py --steps 2 --no-cpu --no-train --no-e2e --no-fusion > gpurun_out/$1_x0.json 2> gpurun_out/$1_x0.err && \
AARMVS_XSPLIT=1 timeout -k 10 300 python bench.py --steps 2 --no-cpu --no-train --no-e2e --no-fusion > gpurun_out/$1_x1b.json 2> gpurun_out/$1_x1b.err
