#!/bin/bash
# Round-6 omega row-sum epilogue: digest + headline A/B (base = the previous commit), the
# 5- and 6-wave builds' headline, then the GPU suite on the in-tree library.
set -o pipefail
T=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_r06_ab.sh $T base notests || exit 1
for w in 5 6; do
  AARMVS_LIB=$PWD/tools/ab/lib_w$w.so timeout -k 10 300 python bench.py --steps 2 --no-cpu --no-train --no-e2e --no-fusion > gpurun_out/${T}_w$w.json 2> gpurun_out/${T}_w$w.err || exit 1
done
python tools/ab_summary.py gpurun_out/${T}_w5.json gpurun_out/${T}_w6.json
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_tests.log
exit $rc
