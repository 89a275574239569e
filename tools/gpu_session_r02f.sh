#!/bin/bash
# Round-2f measurement session: smoke, bench lines (headline with every leg, configs 2 and 5,
# B=2), rocprofv3 kernel stats of the headline command, PMC byte passes (32 planes = two
# plane groups, so per-launch bytes match the headline's 16-plane launches).
source tools/gpu_round.sh
export TMPDIR=/tmp
run smoke 180 python -c "import __graft_entry__ as g; g.smoke()"
run bench_headline 900 python bench.py --train
run bench_cfg2 900 python bench.py --config dtu_eval_800x600_n5_d256 --no-e2e
run bench_cfg5 900 python bench.py --config tnt_1920x1056_n11_d898 --no-e2e --steps 2
run bench_headline_b2 900 python bench.py --batch 2 --no-cpu --no-fusion --no-e2e --steps 2
run prof_stats 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stats -o ks -- python bench.py --no-cpu --no-fusion --no-e2e --steps 2
run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o f -- python bench.py --no-cpu --no-kernel-timing --no-fusion --no-e2e --planes 32 --steps 1 --warmup 0
run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o w -- python bench.py --no-cpu --no-kernel-timing --no-fusion --no-e2e --planes 32 --steps 1 --warmup 0
