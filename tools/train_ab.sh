#!/bin/bash
# A/B of the backward stream schedules on the config-4 training step (AARMVS_BWD_PIPE values,
# alternated): bash tools/train_ab.sh TAG "3 1 3 1" [steps]
set -u
TAG=$1; MODES=$2; STEPS=${3:-3}
mkdir -p gpurun_out
for m in $MODES; do
  AARMVS_BWD_PIPE=$m timeout -k 10 240 python -u tools/train_step.py --steps "$STEPS" > gpurun_out/${TAG}_pipe$m.json 2> gpurun_out/${TAG}_pipe$m.err || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('PIPE', sys.argv[2], d['s_per_step'], d['ms_per_plane'])" gpurun_out/${TAG}_pipe$m.json $m | tee -a gpurun_out/${TAG}_ab.txt
done
