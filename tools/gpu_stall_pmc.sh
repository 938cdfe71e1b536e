#!/bin/bash
# Stall accounting of the persistent run kernels: two SQ passes per
# workload (rocprofv3 --pmc, one counter group per pass, each pass its own time limit):
#   wait:  SQ_WAIT_ANY (parked: s_waitcnt / barrier), SQ_WAIT_INST_ANY (issue stall),
#          SQ_ACTIVE_INST_ANY, SQ_WAVE_CYCLES, SQ_WAIT_INST_LDS, SQ_LDS_BANK_CONFLICT,
#          SQ_LDS_IDX_ACTIVE, SQ_BUSY_CYCLES + GRBM_GUI_ACTIVE
#   issue: SQ_ACTIVE_INST_VALU / _LDS / _SCA / _VMEM / _MISC, SQ_INSTS_VMEM_RD / _WR, SQ_INSTS_SMEM
#          + GRBM_GUI_ACTIVE
# tools/stall_summary.py turns gpurun_out/stall/ into profiles/r06/stall_*.json.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/stall
T=${TAG:-r06}
WAIT="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
ISSUE="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
for cfg in ${CFGS:-4k 4k_vbs}; do
  args="--config $cfg"
  [ $cfg = 4k_vbs ] && args="--config 4k --vbs"
  for grp in wait issue; do
    c="$WAIT"; [ $grp = issue ] && c="$ISSUE"
    timeout -k 10 240 rocprofv3 --pmc $c --output-format csv -d gpurun_out/stall/${T}_${cfg}_$grp -o run -- \
        python3 bench.py $args --steps 1 --warmup 1 --kernel-reps 5 --no-cpu-baseline --no-records --no-pcie \
        --no-parity --detail-out '' > gpurun_out/stall/${T}_${cfg}_$grp.log 2>&1
    rc=$?; echo "pmc $cfg $grp rc=$rc"
    [ $rc -ne 0 ] && { tail -5 gpurun_out/stall/${T}_${cfg}_$grp.log; exit $rc; }
  done
done
exit 0
