#!/bin/bash
# The whole GPU test suite, then smoke(), into gpurun_out/$1_*.log
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$1_tests.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$1_smoke.log 2>&1
