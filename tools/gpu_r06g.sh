#!/bin/bash
# Round-6 step g: the omega-bias gradient's signed error over seeds at two shapes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u tests/diag_omega_bias_seeds.py 8 1 3 32 48 6 > gpurun_out/$1_bias_a.txt 2>&1 || { tail -5 gpurun_out/$1_bias_a.txt; exit 1; }
tail -9 gpurun_out/$1_bias_a.txt
timeout -k 10 500 python -u tests/diag_omega_bias_seeds.py 8 2 4 24 40 5 > gpurun_out/$1_bias_b.txt 2>&1 || { tail -5 gpurun_out/$1_bias_b.txt; exit 1; }
tail -9 gpurun_out/$1_bias_b.txt
