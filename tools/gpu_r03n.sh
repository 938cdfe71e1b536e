#!/bin/bash
# Lone-survivor shortcut + transform-wave priority: parity (large GOP digests) and P-run A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03n; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  timeout -k 10 400 python -u tools/ab_runs.py tools/_ab/noshort.so tools/_ab/prio2.so > $O/ab_$rep.log 2>&1
  rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids $O/ab_$rep.log; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 400 python -u tools/vbs_ab.py tools/_ab/vbscap384.so tools/_ab/vbscap768.so > $O/vbs_ab.log 2>&1
rc=$?; echo "vbs ab rc=$rc"; grep -v amdgpu.ids $O/vbs_ab.log
exit $rc
