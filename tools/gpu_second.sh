#!/bin/bash
source tools/gpu_round.sh
run pytest_gpu 900 python -m pytest tests -m gpu -q
run bench_hl 900 python bench.py --steps 2 --warmup 1 --cpu-planes 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run rocprof_hl 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r1 -o hl --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu
