#!/bin/bash
# Ceiling analysis of the cost-slice kernels (rocprofv3 PMC passes, one counter set per run,
# within the gfx950 per-block limits of MI355X_MICROARCH.md): one 16-plane group of the
# headline sweep (tools/pmc_sweep.py).  Summary: python tools/ceiling_summary.py gpurun_out/ceil
# CEIL_PROG / CEIL_DIR: another driver (e.g. "tools/pmc_fusion.py" for the fusion kernel) and
# output directory.
set -o pipefail
export TMPDIR=/tmp
D=${CEIL_DIR:-gpurun_out/ceil}
PROG=${CEIL_PROG:-tools/pmc_sweep.py --planes 16}
mkdir -p $D
run() {  # run NAME counters...
  local name=$1; shift
  rm -rf $D/$name
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $D/$name -o p -- \
    python3 $PROG > $D/$name.log 2>&1 || { echo "pass $name failed"; tail -3 $D/$name.log; exit 1; }
  echo "pass $name ok"
}
run sq_time SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE
run sq_mix SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
run tex TA_BUSY_avr TA_TOTAL_WAVEFRONTS_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE
run l2 TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_EA0_RDREQ_sum
run fetch FETCH_SIZE
run write WRITE_SIZE
# (CEIL_F64=1) VALU fp64 / transcendental instruction counts and VALU issue
if [ "${CEIL_F64:-0}" = "1" ]; then
  run f64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE
fi
