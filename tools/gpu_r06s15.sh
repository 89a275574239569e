#!/bin/bash
# omega_conv: A = the previous commit (4 items per block), B = in-tree (8 items per block),
# C = the double-buffered box build (tools/ab/lib_db1.so, AARMVS_OMEGA_DB=1) at 8 items per block;
# digests, headline lines A/B/C twice, the parity suites on C, then the GPU suite on B.
set -o pipefail
T=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
A=$PWD/tools/ab/lib_base.so
C=$PWD/tools/ab/lib_db1.so
timeout -k 10 200 python tools/sweep_digest.py > gpurun_out/${T}_digest.txt 2>&1 || exit 1
AARMVS_OMEGA_IPB=8 AARMVS_LIB=$C timeout -k 10 200 python tools/sweep_digest.py >> gpurun_out/${T}_digest.txt 2>&1 || exit 1
grep digest gpurun_out/${T}_digest.txt
for r in 1 2; do
  AARMVS_LIB=$A timeout -k 10 300 python bench.py --steps 2 --no-cpu --no-train --no-e2e --no-fusion > gpurun_out/${T}_A_$r.json 2> gpurun_out/${T}_A_$r.err || exit 1
  timeout -k 10 300 python bench.py --steps 2 --no-cpu --no-train --no-e2e --no-fusion > gpurun_out/${T}_B_$r.json 2> gpurun_out/${T}_B_$r.err || exit 1
  AARMVS_OMEGA_IPB=8 AARMVS_LIB=$C timeout -k 10 300 python bench.py --steps 2 --no-cpu --no-train --no-e2e --no-fusion > gpurun_out/${T}_C_$r.json 2> gpurun_out/${T}_C_$r.err || exit 1
done
python tools/ab_summary.py gpurun_out/${T}_A_1.json gpurun_out/${T}_B_1.json gpurun_out/${T}_C_1.json gpurun_out/${T}_A_2.json gpurun_out/${T}_B_2.json gpurun_out/${T}_C_2.json
AARMVS_LIB=$C timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests_C.log 2>&1 || { tail -3 gpurun_out/${T}_tests_C.log; exit 1; }
tail -1 gpurun_out/${T}_tests_C.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_tests.log
exit $rc
