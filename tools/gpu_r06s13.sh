#!/bin/bash
# omega_conv 16 x 32 haloed tiles (AARMVS_OMEGA_TW=32 build, tools/ab/lib_tw32.so) against the
# library's 16 x 16: digest, headline A/B/A/B, then the parity suites on the 16 x 32 build.
set -o pipefail
T=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
B=$PWD/tools/ab/lib_tw32.so
timeout -k 10 200 python tools/sweep_digest.py > gpurun_out/${T}_digest.txt 2>&1 || exit 1
AARMVS_LIB=$B timeout -k 10 200 python tools/sweep_digest.py >> gpurun_out/${T}_digest.txt 2>&1 || exit 1
cat gpurun_out/${T}_digest.txt | grep digest
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 2 --no-cpu --no-train --no-e2e --no-fusion > gpurun_out/${T}_A_$r.json 2> gpurun_out/${T}_A_$r.err || exit 1
  AARMVS_LIB=$B timeout -k 10 300 python bench.py --steps 2 --no-cpu --no-train --no-e2e --no-fusion > gpurun_out/${T}_B_$r.json 2> gpurun_out/${T}_B_$r.err || exit 1
done
python tools/ab_summary.py gpurun_out/${T}_A_1.json gpurun_out/${T}_B_1.json gpurun_out/${T}_A_2.json gpurun_out/${T}_B_2.json
AARMVS_LIB=$B timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_long.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_tests.log
exit $rc
