#!/bin/bash
# Round-6 step k: the omega-bias error split at test_gpu_bptt's own shapes and seeds (with
# float32's errors), and where seed 104's dL/dx error sits
set -o pipefail
mkdir -p gpurun_out
F32=1 timeout -k 10 900 python -u tests/diag_omega_bias_split.py 17:1,3,32,48,6 16:2,4,24,40,5 29:1,3,16,24,18 > gpurun_out/$1_split_tests.txt 2>&1 || { tail -5 gpurun_out/$1_split_tests.txt; exit 1; }
tail -3 gpurun_out/$1_split_tests.txt
WHERE=1 timeout -k 10 300 python -u tests/diag_omega_bias_split.py 104 100 > gpurun_out/$1_split_where.txt 2>&1
tail -4 gpurun_out/$1_split_where.txt
