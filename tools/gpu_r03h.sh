#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03h; mkdir -p $O
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for v in default phase1 phase2; do
  if [ $v = default ]; then unset SO_LIB_PATH; else export SO_LIB_PATH=tools/_ab/$v.so; fi
  timeout -k 10 120 python tools/prun_phase.py --vbs --reps 6 > $O/time_vbs_$v.log 2>&1
  rc=$?; echo "time $v rc=$rc: $(tail -1 $O/time_vbs_$v.log)"; [ $rc -ne 0 ] && exit $rc
  timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/pmc_vbs_$v -o run -- python3 tools/prun_phase.py --vbs --reps 2 \
      > $O/pmc_vbs_$v.log 2>&1
  rc=$?; echo "pmc $v rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
