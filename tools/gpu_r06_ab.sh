#!/bin/bash
# Round-6 A/B: sweep digest of tools/ab/lib_$2.so (A) and the in-tree library (B), the headline
# bench A/B/A/B (kernel timing, no CPU leg), then the GPU test suite on the in-tree library.
# usage: bash tools/gpu_r06_ab.sh TAG LIBTAG [notests]
set -o pipefail
mkdir -p gpurun_out
T=$1
A=$PWD/tools/ab/lib_$2.so
export TMPDIR=/tmp
AARMVS_LIB=$A timeout -k 10 200 python tools/sweep_digest.py > gpurun_out/${T}_digest.txt 2>&1 || exit 1
timeout -k 10 200 python tools/sweep_digest.py >> gpurun_out/${T}_digest.txt 2>&1 || exit 1
cat gpurun_out/${T}_digest.txt
for r in 1 2; do
  AARMVS_LIB=$A timeout -k 10 300 python bench.py --steps 2 --no-cpu --no-train --no-e2e --no-fusion > gpurun_out/${T}_A_$r.json 2> gpurun_out/${T}_A_$r.err || exit 1
  timeout -k 10 300 python bench.py --steps 2 --no-cpu --no-train --no-e2e --no-fusion > gpurun_out/${T}_B_$r.json 2> gpurun_out/${T}_B_$r.err || exit 1
done
python tools/ab_summary.py gpurun_out/${T}_A_1.json gpurun_out/${T}_B_1.json gpurun_out/${T}_A_2.json gpurun_out/${T}_B_2.json
if [ "${3:-}" != "notests" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
  rc=$?
  tail -3 gpurun_out/${T}_tests.log
  exit $rc
fi
