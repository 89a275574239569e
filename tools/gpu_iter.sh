#!/bin/bash
# tests + headline bench (kernel timing on)
source tools/gpu_round.sh
run pytest_gpu 900 python -m pytest tests -m gpu -q -x
run bench_hl 900 python bench.py --steps 2 --warmup 1 --no-cpu
