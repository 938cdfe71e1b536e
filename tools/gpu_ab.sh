#!/bin/bash
# Interleaved P-run A/B (tools/ab_interleave.py) after the GPU parity suite on the default build.
#   AB="default tools/_ab/x.so" TAG=name ROUNDS=3 PYTEST=1 tools/gpu_ab.sh
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ab}; mkdir -p $O
if [ "${PYTEST:-1}" = 1 ]; then
  timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread \
      -p no:cacheprovider > $O/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 900 python -u tools/ab_interleave.py --rounds ${ROUNDS:-3} $AB > $O/ab.log 2>&1
rc=$?; echo "ab rc=$rc"; grep summary $O/ab.log; [ $rc -ne 0 ] && tail -5 $O/ab.log
exit $rc
