#!/bin/bash
# VBS persistent run with the exact block + sub-block SEA: parity, A/B against the dense search,
# the 4K VBS bench.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03g; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_pipeline.py -x -q -m gpu --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "vbs" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR|Error" $O/pytest.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/vbs_ab.py tools/_ab/vbsdense.so > $O/vbs_ab.log 2>&1
rc=$?; echo "ab rc=$rc"; cat $O/vbs_ab.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --vbs --steps 10 --warmup 2 --no-cpu-baseline --no-pcie > $O/bench_vbs.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"bit_exact": [a-z]*' $O/bench_vbs.log | head -3 | tr '\n' ' '; echo
exit $rc
