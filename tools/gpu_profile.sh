#!/bin/bash
# Round profile: default bench line (with CPU baseline), rocprofv3 kernel stats of the
# same command (tools/prof_lastpass.py picks out its serialised kernel-timing pass), and the FETCH_SIZE / WRITE_SIZE passes (short sweep: per-launch bytes)
source tools/gpu_round.sh
export TMPDIR=/tmp
run bench_default 900 python bench.py
run prof_stats 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stats -o ks -- python bench.py --no-cpu
run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o f -- python bench.py --no-cpu --no-kernel-timing --planes 8 --steps 1 --warmup 0
run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o w -- python bench.py --no-cpu --no-kernel-timing --planes 8 --steps 1 --warmup 0
