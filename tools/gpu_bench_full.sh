#!/bin/bash
# The default bench line (what the driver runs at round end) into gpurun_out/$1.json
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python bench.py > gpurun_out/$1.json 2> gpurun_out/$1.err
