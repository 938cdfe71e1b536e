#!/bin/bash
# PMC passes over tools/frame_one.py (4K P-frame ME+TQ and an I-frame, 5 times each):
#   sq1/sq2: issue and stall counters of every kernel
#   fetch / write: FETCH_SIZE and WRITE_SIZE in separate passes (they do not fit one pass)
# Parsed on the host by tools/pmc_summary.py into profiles/.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
TAG=${1:-r01}
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
SQ2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
run() {  # name, counters
  timeout -k 10 300 rocprofv3 --pmc $2 --output-format csv -d gpurun_out/pmc/${TAG}_$1 -o run -- \
      python3 tools/frame_one.py > gpurun_out/pmc/${TAG}_$1.log 2>&1
  local rc=$?; echo "pmc $1 rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc/${TAG}_$1.log; exit $rc; }
  return 0
}
run sq1 "$SQ1"
run sq2 "$SQ2"
run fetch "FETCH_SIZE"
run write "WRITE_SIZE"
ls gpurun_out/pmc/
