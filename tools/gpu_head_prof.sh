#!/bin/bash
# rocprofv3 kernel statistics of the headline bench command (the roofline's kernel average
# must agree with bench.py's hipEvent figure) -> gpurun_out/$1/
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$1 -o run -- \
  python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-train --no-e2e --no-fusion > $R/gpurun_out/$1.json 2> $R/gpurun_out/$1.err
