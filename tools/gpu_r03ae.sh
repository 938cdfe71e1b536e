#!/bin/bash
# PMC passes over the 4K P-run (tools/prun_phase.py, 3 launches), plain and VBSEnable:
# issue counters, stall / LDS counters
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03ae; mkdir -p $O
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
SQ2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
run() {  # name, counters, args
  timeout -s KILL 120 rocprofv3 --pmc $2 --output-format csv -d $O/$1 -o run -- python3 tools/prun_phase.py --reps 3 $3 > $O/$1.log 2>&1
  local rc=$?; echo "pmc $1 rc=$rc"; [ $rc -ne 0 ] && { tail -3 $O/$1.log; exit $rc; }; return 0
}
run plain_sq1 "$SQ1" "" && run plain_sq2 "$SQ2" "" && run vbs_sq1 "$SQ1" "--vbs" && run vbs_sq2 "$SQ2" "--vbs"
