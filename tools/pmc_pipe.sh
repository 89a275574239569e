#!/bin/bash
# memory-pipe counter passes over the pipeline microbench (one rocprofv3 --pmc pass per group)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE GRBM_TA_BUSY TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum \
  --output-format csv -d gpurun_out/pmc_pipe3 -o p3 -- ./tools/microbench/pipe_bench > gpurun_out/pmc_pipe3.log 2>&1
echo rc=$?
