#!/bin/bash
# Round-6 step j: split the omega-bias gradient's GPU error into the BPTT's (dL/dx) share and the
# cost-slice backward's own, at the seeds of tests/diag_omega_bias_seeds.py
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u tests/diag_omega_bias_split.py 104 102 100 103 > gpurun_out/$1_split.txt 2>&1
rc=$?
tail -6 gpurun_out/$1_split.txt
exit $rc
