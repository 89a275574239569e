#!/bin/bash
# End-of-round evidence on one box: rocprofv3 kernel statistics of the headline bench
# (gpu_head_prof.sh), the PMC ceiling passes (gpu_ceiling.sh), then the default bench line.
# bash tools/gpu_final_prof.sh TAG
set -o pipefail
T=$1
mkdir -p gpurun_out
bash tools/gpu_head_prof.sh ${T}_head || exit 1
CEIL_DIR=gpurun_out/ceil_$T bash tools/gpu_ceiling.sh > gpurun_out/ceil_$T.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench_default.json 2> gpurun_out/${T}_bench_default.err
