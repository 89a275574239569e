#!/bin/bash
# MFMA-pipe utilisation of the sweep's kernels (rocprofv3 PMC pass, 8 planes of the headline
# sweep, serialised kernel-timing pass included): SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES,
# GRBM_GUI_ACTIVE, SQ_INSTS_VALU, SQ_INSTS_MFMA
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/pmc_mfma
timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA \
  --output-format csv -d gpurun_out/pmc_mfma -o m -- python bench.py --no-cpu --no-fusion --no-e2e --no-train --planes 8 \
  --steps 1 --warmup 0 > gpurun_out/pmc_mfma.log 2>&1 || { tail -5 gpurun_out/pmc_mfma.log; exit 1; }
python tools/pmc_show.py gpurun_out/pmc_mfma lstm omega cost_x deconv head
