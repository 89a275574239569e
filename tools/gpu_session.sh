#!/bin/bash
# Measurement session: all GPU tests + smoke, bench lines (headline, configs 2 and 5,
# batched headline), rocprofv3 kernel stats of the headline command, PMC bytes passes.
source tools/gpu_round.sh
export TMPDIR=/tmp
run tests 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread
run smoke 180 python -c "import __graft_entry__ as g; g.smoke()"
run bench_headline 900 python bench.py --train
run bench_cfg2 900 python bench.py --config dtu_eval_800x600_n5_d256 --no-e2e
run bench_cfg5 900 python bench.py --config tnt_1920x1056_n11_d898 --no-e2e --steps 2
run bench_headline_b2 900 python bench.py --batch 2 --no-cpu --no-fusion --no-e2e --steps 2
run prof_stats 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stats -o ks -- python bench.py --no-cpu --no-fusion --no-e2e --steps 2
run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o f -- python bench.py --no-cpu --no-kernel-timing --no-fusion --no-e2e --planes 8 --steps 1 --warmup 0
run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o w -- python bench.py --no-cpu --no-kernel-timing --no-fusion --no-e2e --planes 8 --steps 1 --warmup 0
