#!/bin/bash
# SQ / TA counters for omega_conv vs omega_strip (4 planes of the headline sweep)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for var in valu strip; do
  for pass in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES" \
              "TA_BUSY_avr TA_BUFFER_READ_WAVEFRONTS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE"; do
    tag=$(echo $pass | cut -c1-6)
    AARMVS_OMEGA=$var AB_OUT=/tmp/pmc_$var.npy timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv \
      -d gpurun_out/pmc_strip_${var}_$tag -o p -- python tools/variant_ab.py --child --planes 4 \
      > gpurun_out/pmc_strip_${var}_$tag.log 2>&1 || { echo "FAIL $var $tag"; tail -5 gpurun_out/pmc_strip_${var}_$tag.log; exit 1; }
    python tools/pmc_show.py gpurun_out/pmc_strip_${var}_$tag omega_conv omega_strip cost_x
  done
done
