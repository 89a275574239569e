#!/bin/bash
# Round-6 final evidence, part A: the GPU suite, smoke(), rocprofv3 kernel statistics of the
# headline bench, the PMC ceiling passes (traffic + limiters of the final tree).
set -o pipefail
T=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -20 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -5 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
bash tools/gpu_head_prof.sh ${T}_head || exit 1
CEIL_DIR=gpurun_out/ceil_$T bash tools/gpu_ceiling.sh > gpurun_out/ceil_$T.log 2>&1 || { tail -5 gpurun_out/ceil_$T.log; exit 1; }
python tools/ceiling_summary.py gpurun_out/ceil_$T --out gpurun_out/${T}_ceiling_pmc.json > /dev/null 2>&1
python tools/pmc_summarize.py gpurun_out/ceil_$T/fetch gpurun_out/ceil_$T/write --workload dtu_eval_1600x1184_n7_d512 --source "round 6 final tree ($T): tools/gpu_ceiling.sh fetch/write passes over one 16-plane group at the headline" --out gpurun_out/${T}_pmc_traffic.json > gpurun_out/${T}_pmc_traffic.txt 2>&1
ls gpurun_out/${T}_head
