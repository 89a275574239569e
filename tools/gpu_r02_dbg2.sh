#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python tools/variant_ab.py --planes 12 AARMVS_OMEGA=valu AARMVS_OMEGA=valu,AB_OVERLAP=0 \
  AARMVS_OMEGA=mfma AARMVS_OMEGA=mfma,AB_OVERLAP=0 AARMVS_OMEGA=mfma,AARMVS_PIPE_BOX_CAP=4 \
  AARMVS_OMEGA=mfma,AARMVS_PIPE_BOX_CAP=4,AB_OVERLAP=0 > gpurun_out/r02_dbg2.log 2>&1; rc=$?
cut -c1-400 gpurun_out/r02_dbg2.log
exit $rc
