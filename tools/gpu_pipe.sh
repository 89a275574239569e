#!/bin/bash
# pipeline microbenchmark only (omega_conv / cost_x variants)
source tools/gpu_round.sh
run pipe_bench 120 ./tools/microbench/pipe_bench
