#!/bin/bash
# intra recon as a chunked scan: GPU suite, I-frame A/B against the sequential walk, kernel times
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03w}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/intra_ab.py tools/_ab/wpr8.so tools/_ab/wpr16.so "" tools/_ab/wpr8.so tools/_ab/wpr16.so > $O/intra_ab.log 2>&1
rc=$?; echo "intra_ab rc=$rc"; cat $O/intra_ab.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 tools/intra_ab.py > $GRAFT_REPO_ROOT/$O/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
