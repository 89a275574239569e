#!/bin/bash
# fusion tests + full GPU test suite + bench with the fusion leg
source tools/gpu_round.sh
run pytest_fusion 300 python -u -m pytest tests/test_fusion.py -m gpu -x -v --timeout 120 --timeout-method thread
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run bench_hl 900 python bench.py
