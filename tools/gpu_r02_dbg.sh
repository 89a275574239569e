#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/debug_omega.py 1184 1600 7 > gpurun_out/r02_dbg.log 2>&1; rc=$?
cat gpurun_out/r02_dbg.log | grep -v Warning | tail -30
exit $rc
