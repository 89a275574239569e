#!/bin/bash
# Round-2 GPU validation: every -m gpu test, smoke(), one headline bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  > gpurun_out/r02_tests.log 2>&1 || { echo "TESTS FAILED rc=$?"; tail -40 gpurun_out/r02_tests.log; exit 1; }
tail -5 gpurun_out/r02_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_smoke.log 2>&1 || { echo SMOKE FAILED; cat gpurun_out/r02_smoke.log; exit 1; }
cat gpurun_out/r02_smoke.log
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/r02_bench.log 2>&1 || { echo BENCH FAILED; tail -30 gpurun_out/r02_bench.log; exit 1; }
tail -c 3000 gpurun_out/r02_bench.log
