#!/bin/bash
# Headline-metric lines for the other BASELINE configs and B=2 (parity sections skipped)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config dtu_eval_800x600_n5_d256 --no-cpu --no-train --no-e2e --no-fusion --no-kernel-timing > gpurun_out/$1_cfg2.json 2> gpurun_out/$1_cfg2.err && \
timeout -k 10 400 python bench.py --config tnt_1920x1056_n11_d898 --steps 2 --no-cpu --no-train --no-e2e --no-fusion > gpurun_out/$1_cfg5.json 2> gpurun_out/$1_cfg5.err && \
timeout -k 10 300 python bench.py --batch 2 --steps 2 --no-cpu --no-train --no-e2e --no-fusion --no-kernel-timing > gpurun_out/$1_b2.json 2> gpurun_out/$1_b2.err && \
timeout -k 10 200 python bench.py --config plumbing_160x128_n3_d48 --steps 20 --warmup 3 --no-train --no-e2e --no-fusion --no-kernel-timing > gpurun_out/$1_cfg1.json 2> gpurun_out/$1_cfg1.err
