#!/bin/bash
# Round-6 step c: the 4x4x4 MFMA layout probe, then the A/B of tools/gpu_r06_ab.sh
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/microbench/mfma4_layout > gpurun_out/$1_mfma4_layout.txt 2>&1; rc=$?
cat gpurun_out/$1_mfma4_layout.txt | head -5
[ $rc -le 1 ] || exit $rc
bash tools/gpu_r06_ab.sh "$@"
