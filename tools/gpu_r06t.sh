#!/bin/bash
# Round-6 step t: the training record's omega conv output and statistics written / read in place
# (no copies) -- the training tests, then the training step
set -o pipefail
mkdir -p gpurun_out
T=$1
timeout -k 10 900 python -u -m pytest tests/test_gpu_bptt.py tests/test_gpu_training.py tests/test_gpu_train_fixtures.py -x -q --timeout 400 --timeout-method thread \
  > gpurun_out/${T}_tests.log 2>&1 || { tail -20 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --train --steps 6 --warmup 2 --no-cpu --no-kernel-timing > gpurun_out/${T}_t$i.json 2> gpurun_out/${T}_t$i.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/${T}_t$i.json').read().strip().split('\n')[-1]); print(d['value'], d['ms_per_step'])"
done
