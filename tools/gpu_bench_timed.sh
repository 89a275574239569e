#!/bin/bash
# The driver's default bench command, timed, into gpurun_out/$1.json (+ wall seconds in $1.time)
set -o pipefail
mkdir -p gpurun_out
s=$(date +%s)
timeout -k 10 1000 python bench.py > gpurun_out/$1.json 2> gpurun_out/$1.err || exit 1
echo $(( $(date +%s) - s )) > gpurun_out/$1.time
