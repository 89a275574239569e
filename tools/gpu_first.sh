#!/bin/bash
source tools/gpu_round.sh
rocm-smi --showproductname > gpurun_out/smi.log 2>&1 || true
run pytest_gpu 900 python -m pytest tests -m gpu -x -q
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench_dtu 600 python bench.py --config dtu_eval_800x600_n5_d256 --steps 2 --warmup 1 --cpu-planes 1
run bench_dtu_nt 600 python bench.py --config dtu_eval_800x600_n5_d256 --steps 2 --warmup 1 --no-cpu --no-kernel-timing
