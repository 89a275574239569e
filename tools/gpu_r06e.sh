#!/bin/bash
# Round-6 step e: A/B (digest, headline x2) against tools/ab/lib_$2.so, then the in-tree library
# at omega items-per-block 2 and 8, then the GPU test suite.
set -o pipefail
T=$1
bash tools/gpu_r06_ab.sh $T $2 notests || exit 1
for n in 2 8; do
  AARMVS_OMEGA_IPB=$n timeout -k 10 300 python bench.py --steps 2 --no-cpu --no-train --no-e2e --no-fusion > gpurun_out/${T}_ipb$n.json 2> gpurun_out/${T}_ipb$n.err || exit 1
done
python tools/ab_summary.py gpurun_out/${T}_ipb2.json gpurun_out/${T}_ipb8.json
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_tests.log
exit $rc
