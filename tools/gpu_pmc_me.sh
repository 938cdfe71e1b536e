#!/bin/bash
# PMC passes over tools/me_one.py (4K P-frame ME only) for each ME implementation.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcme
TAG=${1:-me}
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_SMEM SQ_INST_CYCLES_SMEM"
P3="SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_IFETCH SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE"
for impl in ${IMPLS:-sea dense}; do
  for p in 1 2 3; do
    eval "ctrs=\$P$p"
    SO_ME_IMPL=$impl ME_N=5 timeout -k 10 300 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/pmcme/${TAG}_${impl}_p$p -o run -- python3 tools/me_one.py > gpurun_out/pmcme/${TAG}_${impl}_p$p.log 2>&1
    rc=$?; echo "pmc $impl p$p rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmcme/${TAG}_${impl}_p$p.log; exit $rc; }
  done
done
