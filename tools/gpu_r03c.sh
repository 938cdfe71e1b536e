#!/bin/bash
# p_run_kernel phase attribution: timing + SQ counters of the product build and of the builds
# with the transforms (phase1) or the search (phase2) compiled out; the full-frame CPU timing
# of BASELINE.md section 3 runs beside it on the host.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03c; mkdir -p $O
timeout -k 10 900 python tools/cpu_full_frame.py > $O/cpu_full_frame.json 2> $O/cpu_full_frame.err &
CPU_PID=$!
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for v in default phase1 phase2; do
  if [ $v = default ]; then unset SO_LIB_PATH; else export SO_LIB_PATH=tools/_ab/$v.so; fi
  timeout -k 10 120 python tools/prun_phase.py --reps 10 > $O/time_$v.log 2>&1
  rc=$?; echo "time $v rc=$rc: $(tail -1 $O/time_$v.log)"; [ $rc -ne 0 ] && exit $rc
  timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/pmc_$v -o run -- python3 tools/prun_phase.py --reps 2 \
      > $O/pmc_$v.log 2>&1
  rc=$?; echo "pmc $v rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
unset SO_LIB_PATH
wait $CPU_PID
echo "cpu rc=$?: $(cat $O/cpu_full_frame.json)"
exit 0
