#!/bin/bash
# parity tests + pipeline microbench
source tools/gpu_round.sh
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run pipe_bench 120 ./tools/microbench/pipe_bench
