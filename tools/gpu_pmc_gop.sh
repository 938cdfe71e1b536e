#!/bin/bash
# SQ counter passes over tools/frame_gop.py (4K P-frame ME + TQ on the GOP's real reference).
# Summarised on the host by tools/pmc_gop_table.py.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-gop}
OUT=gpurun_out/pmcgop
mkdir -p $OUT
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS"
P3="SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_LDS SQ_LDS_ADDR_CONFLICT SQ_IFETCH SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
for p in 1 2 3; do
  eval "ctrs=\$P$p"
  timeout -k 10 120 rocprofv3 --pmc $ctrs --output-format csv -d $OUT/${TAG}_p$p -o run -- python3 tools/frame_gop.py > $OUT/${TAG}_p$p.log 2>&1
  rc=$?; echo "pmc p$p rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/${TAG}_p$p.log; exit $rc; }
done
exit 0
