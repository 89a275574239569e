#!/bin/bash
# Round-6 final evidence, part B: the default bench line (CPU baseline, fusion, e2e, training),
# then the other configs' lines (tools/gpu_configs.sh).
set -o pipefail
T=$1
mkdir -p gpurun_out
timeout -k 10 700 python -u bench.py > gpurun_out/${T}_bench_default.json 2> gpurun_out/${T}_bench_default.err || { tail -5 gpurun_out/${T}_bench_default.err; exit 1; }
cut -c1-400 gpurun_out/${T}_bench_default.json
bash tools/gpu_configs.sh $T || exit 1
for f in gpurun_out/${T}_cfg1.json gpurun_out/${T}_cfg2.json gpurun_out/${T}_cfg5.json gpurun_out/${T}_b2.json; do cut -c1-200 $f; done
