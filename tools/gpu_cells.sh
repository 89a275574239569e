#!/bin/bash
# tests + cell microbench + headline bench
source tools/gpu_round.sh
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run cell_bench 200 ./tools/microbench/cell_bench
run bench_hl 600 python bench.py --steps 2 --warmup 1 --no-cpu
