#!/bin/bash
source tools/gpu_round.sh
run pytest_gpu 900 python -m pytest tests -m gpu -q -x
run pipe_bench 200 ./tools/microbench/pipe_bench
