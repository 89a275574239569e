#!/bin/bash
# omega_conv / cost_x: pipeline microbench ablations + two SQ counter passes
source tools/gpu_round.sh
export TMPDIR=/tmp
run pipe_bench 120 ./tools/microbench/pipe_bench
run pmc_sq1 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --output-format csv -d gpurun_out/pmc_sq1 -o s1 -- ./tools/microbench/pipe_bench
run pmc_sq2 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_UNALIGNED_STALL --output-format csv -d gpurun_out/pmc_sq2 -o s2 -- ./tools/microbench/pipe_bench
