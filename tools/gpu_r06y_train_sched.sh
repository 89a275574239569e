#!/bin/bash
# Round-6: the training step's stream schedules with the shared library streams -- backward
# pipeline AARMVS_BWD_PIPE 1 (default) / 3 / 0 and the recorded forward on 3 / 2 unit streams,
# interleaved twice on one box
set -o pipefail
mkdir -p gpurun_out
T=$1
for r in 1 2; do
  for cfg in "1 3" "3 3" "0 3" "1 2"; do
    set -- $cfg
    AARMVS_BWD_PIPE=$1 AARMVS_REG_STREAMS_REC=$2 timeout -k 10 300 python -u bench.py --train --steps 6 --warmup 2 --no-cpu --no-kernel-timing \
      > gpurun_out/${T}_p$1_r$2_$r.json 2> gpurun_out/${T}_p$1_r$2_$r.err || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); print(sys.argv[1].split('/')[-1], d['ms_per_step'], 'ms')" gpurun_out/${T}_p$1_r$2_$r.json
  done
done | tee gpurun_out/${T}_summary.txt
