#!/bin/bash
# SEA survivor cap A/B, the no-transform phase build (timing + SQ counters), and the per-tile
# phase stamps of the p_run kernel at 4K and 1088p.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03d; mkdir -p $O
timeout -k 10 300 python tools/ab_runs.py tools/_ab/cap256.so tools/_ab/cap384.so > $O/ab_cap.log 2>&1
rc=$?; echo "ab rc=$rc"; cat $O/ab_cap.log; [ $rc -ne 0 ] && exit $rc
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
export SO_LIB_PATH=tools/_ab/phase1.so
timeout -k 10 120 python tools/prun_phase.py --reps 10 > $O/time_phase1.log 2>&1
rc=$?; echo "time phase1 rc=$rc: $(tail -1 $O/time_phase1.log)"; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/pmc_phase1 -o run -- python3 tools/prun_phase.py --reps 2 \
    > $O/pmc_phase1.log 2>&1
rc=$?; echo "pmc phase1 rc=$rc"; [ $rc -ne 0 ] && exit $rc
export SO_LIB_PATH=tools/_ab/stamps.so
timeout -k 10 200 python tools/run_stamps.py --heights 1088,2160 > $O/stamps.log 2>&1
rc=$?; echo "stamps rc=$rc"; tail -c 3000 $O/stamps.log
exit $rc
