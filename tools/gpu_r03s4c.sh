#!/bin/bash
# The 32-bit sub-block key variant (tools/patches/vbs_keys32.patch, built as tools/_ab/keys32.so):
# the VBS GPU tests through it, then the VBS P-run A/B against the product build, interleaved twice.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03s4c; mkdir -p $O
SO_LIB_PATH=tools/_ab/keys32.so timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "vbs or VBS" --timeout 300 \
    --timeout-method thread -p no:cacheprovider > $O/pytest_gpu_keys32.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" $O/pytest_gpu_keys32.log | tail -4; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  timeout -k 10 400 python -u tools/vbs_ab.py tools/_ab/keys32.so >> $O/vbs_ab.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "vbs_ab rc=$rc"; tail -5 $O/vbs_ab.log; exit $rc; }
done
cat $O/vbs_ab.log
