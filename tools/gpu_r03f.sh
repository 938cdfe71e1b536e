#!/bin/bash
# VBSEnable in the persistent run: parity tests, then the 4K VBS bench and its kernel trace.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03f; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_pipeline.py -x -q -m gpu --timeout 300 \
    --timeout-method thread -p no:cacheprovider -k "vbs or two_processes" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR|Error" $O/pytest.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --vbs --steps 10 --warmup 2 --no-cpu-baseline --no-pcie > $O/bench_vbs.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"bit_exact": [a-z]*' $O/bench_vbs.log | head -3 | tr '\n' ' '; echo
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_vbs -o run -- \
    python3 bench.py --vbs --steps 3 --warmup 1 --no-cpu-baseline --no-pcie --no-parity > $O/prof_vbs.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
