#!/bin/bash
# Round-6 step m: the float64 backward tests (omega bias: common bound or 1/2 u sum|terms|), then
# the training step with the recorded forward's regulariser on 1 or 3 streams, with the default
# 4 hardware queues per process and with 8 (is the 3-stream slowdown queue sharing?)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bptt.py -x -v -s --timeout 400 --timeout-method thread \
  -k "float64 or systematic" > gpurun_out/$1_bptt.log 2>&1 || { grep -E "passed|failed|Error" gpurun_out/$1_bptt.log; exit 1; }
grep -E "passed|failed|u sum" gpurun_out/$1_bptt.log
out=gpurun_out/$1_train_streams.txt
: > $out
for rq in "1 4" "3 4" "1 8" "3 8" "2 4"; do
  set -- $rq "$1"
  echo "REG_STREAMS_REC=$1 GPU_MAX_HW_QUEUES=$2" | tee -a $out
  AARMVS_REG_STREAMS_REC=$1 GPU_MAX_HW_QUEUES=$2 timeout -k 10 300 python -u bench.py --train --steps 6 --warmup 2 \
    --no-cpu --no-kernel-timing > gpurun_out/$3_train_$1_$2.json 2> gpurun_out/$3_train_$1_$2.err || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['value'])" \
    gpurun_out/$3_train_$1_$2.json | tee -a $out
  set -- "$3"
done
