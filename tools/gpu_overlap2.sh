#!/bin/bash
source tools/gpu_round.sh
run pytest_gpu 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread
run b_costx 600 python bench.py --no-cpu --no-kernel-timing --no-fusion
AARMVS_OVERLAP=all run b_all 600 python bench.py --no-cpu --no-kernel-timing --no-fusion
run b_single 600 python bench.py --no-cpu --no-kernel-timing --no-fusion --no-overlap
