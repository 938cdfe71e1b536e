#!/bin/bash
# PMC passes (issue / stall counters) of the P-run for several library variants:
#   VARIANTS="default tools/_ab/x.so" SO_AB_VBS=1 TAG=name tools/gpu_pmc_variants.sh
# Summarised on the host by tools/pmc_variants.py.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pmcv}; mkdir -p $O
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
SQ2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
for v in $VARIANTS; do
  n=$(basename $v .so)
  lib=""; [ "$v" != default ] && lib=$v
  for p in sq1 sq2; do
    c=$SQ1; [ $p = sq2 ] && c=$SQ2
    SO_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/${n}_$p -o run -- \
        python3 tools/prun_one.py > $O/${n}_$p.log 2>&1
    rc=$?; echo "pmc $n $p rc=$rc"
    [ $rc -ne 0 ] && { tail -5 $O/${n}_$p.log; exit $rc; }
  done
done
exit 0
