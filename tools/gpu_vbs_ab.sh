#!/bin/bash
# VBS round-5 A/B: the GPU suite on the default build, the VBS tests on each variant library,
# then the interleaved VBS P-run A/B (tools/ab_interleave.py, SO_AB_VBS=1).
#   VARIANTS="tools/_ab/a.so tools/_ab/b.so" TAG=name tools/gpu_vbs_ab.sh
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-vbsab}; mkdir -p $O
if [ "${PYTEST:-1}" = 1 ]; then
  timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread \
      -p no:cacheprovider > $O/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
fi
for v in $VARIANTS; do
  n=$(basename $v .so)
  SO_LIB_PATH=$v timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "vbs or VBS" --timeout 120 \
      --timeout-method thread -p no:cacheprovider > $O/pytest_$n.log 2>&1
  rc=$?; echo "pytest[$n] rc=$rc"; tail -1 $O/pytest_$n.log; [ $rc -ne 0 ] && exit $rc
done
SO_AB_VBS=1 timeout -k 10 900 python -u tools/ab_interleave.py --rounds ${ROUNDS:-3} ${BASE:-tools/_ab/base.so} default $VARIANTS > $O/ab.log 2>&1
rc=$?; echo "ab rc=$rc"; grep summary $O/ab.log; [ $rc -ne 0 ] && tail -5 $O/ab.log
exit $rc
