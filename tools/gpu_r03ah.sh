#!/bin/bash
# intra scan rows grouped per XCD: GPU suite, I-frame A/B, kernel times and HBM bytes
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03ah; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/intra_ab.py tools/_ab/head.so "" tools/_ab/head.so > $O/intra_ab.log 2>&1
rc=$?; echo "intra_ab rc=$rc"; cat $O/intra_ab.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/intra_ab.py > $O/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$c -o run -- python3 tools/intra_ab.py > $O/pmc_$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
