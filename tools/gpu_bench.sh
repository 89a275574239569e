#!/bin/bash
# parity tests + headline bench (no CPU baseline)
source tools/gpu_round.sh
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run bench_hl 600 python bench.py --no-cpu
