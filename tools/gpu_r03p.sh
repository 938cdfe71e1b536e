#!/bin/bash
# Stall attribution of p_run_kernel (4K P-run of the bench GOP, tools/prun_phase.py): where the
# VALU-idle third of the cycles goes (s_waitcnt / barrier parking vs issue stalls vs LDS).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03p; mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE"
P3="SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_INST_LEVEL_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -k 10 120 python -u tools/prun_phase.py --reps 5 > $O/time.log 2>&1
rc=$?; echo "time rc=$rc"; grep -v amdgpu.ids $O/time.log | tail -2; [ $rc -ne 0 ] && exit $rc
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o run -- \
      python3 tools/prun_phase.py --reps 2 > $O/p$i.log 2>&1
  rc=$?; echo "pmc p$i rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/p$i.log; exit $rc; }
done
exit 0
