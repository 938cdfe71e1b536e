#!/bin/bash
# VBS P-run phase attribution: issue counters with the transforms compiled out (phase1) and
# with the search compiled out (phase2), plus their times
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03af; mkdir -p $O
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
for ph in 1 2; do
  SO_LIB_PATH=tools/_ab/phase$ph.so timeout -k 10 120 python3 tools/prun_phase.py --vbs --reps 5 > $O/time_phase$ph.log 2>&1
  rc=$?; echo "time phase$ph rc=$rc"; grep '^{' $O/time_phase$ph.log; [ $rc -ne 0 ] && exit $rc
  SO_LIB_PATH=tools/_ab/phase$ph.so timeout -s KILL 120 rocprofv3 --pmc $SQ1 --output-format csv -d $O/vbs_phase$ph -o run -- python3 tools/prun_phase.py --vbs --reps 3 > $O/vbs_phase$ph.log 2>&1
  rc=$?; echo "pmc phase$ph rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
