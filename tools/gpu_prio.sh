source tools/gpu_round.sh
run b_default 600 python bench.py --no-cpu --no-kernel-timing
run b_prio 600 python bench.py --no-cpu --no-kernel-timing --high-priority
run b_single 600 python bench.py --no-cpu --no-kernel-timing --no-overlap
