#!/bin/bash
# headline bench line with the end-to-end leg (no CPU baseline, no fusion)
source tools/gpu_round.sh
run bench_e2e 600 python bench.py --no-cpu --no-fusion
