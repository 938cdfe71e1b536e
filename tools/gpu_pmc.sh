#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 120 ./tools/ubench_sad > gpurun_out/ubench_sad.log 2>&1; rc=$?; echo "ubench rc=$rc"; cat gpurun_out/ubench_sad.log
[ $rc -ne 0 ] && exit $rc
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU"
for impl in sad qsad; do
  for p in 1 2; do
    eval "ctrs=\$P$p"
    SO_ME_IMPL=$impl timeout -k 10 300 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/pmc/${impl}_p$p -o run -- python3 tools/me_one.py > gpurun_out/pmc/${impl}_p$p.log 2>&1
    rc=$?; echo "pmc $impl p$p rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc/${impl}_p$p.log; exit $rc; }
  done
done
ls -R gpurun_out/pmc | head -30
