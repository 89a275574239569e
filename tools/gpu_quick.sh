#!/bin/bash
# parity tests + pipeline and cell microbenches
source tools/gpu_round.sh
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run pipe_bench 120 ./tools/microbench/pipe_bench
run cell_bench 120 ./tools/microbench/cell_bench
