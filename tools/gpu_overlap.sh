#!/bin/bash
source tools/gpu_round.sh
run pytest_gpu 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread
run b_ovl 300 python bench.py --steps 2 --warmup 1 --no-cpu --no-kernel-timing
run b_noovl 300 python bench.py --steps 2 --warmup 1 --no-cpu --no-kernel-timing --no-overlap
run b_hp 300 python bench.py --steps 2 --warmup 1 --no-cpu --no-kernel-timing --high-priority
