#!/bin/bash
# One-task-ahead prefetch in the P-run: the 4K digest test alone first, then the suite, then A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03t; mkdir -p $O
timeout -k 10 200 python -u -m pytest "tests/test_gpu_large.py::test_benchmarked_gop_bit_exact" -x -v --timeout 150 \
    --timeout-method thread -p no:cacheprovider > $O/pytest_4k.log 2>&1
rc=$?; echo "pytest 4k rc=$rc"; tail -4 $O/pytest_4k.log; [ $rc -ne 0 ] && exit $rc
AB="default tools/_ab/nopf.so" TAG=r03t ROUNDS=3 tools/gpu_ab.sh
