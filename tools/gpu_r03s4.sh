#!/bin/bash
# Session 4: the GPU suite on the current build, the VBS P-run A/B (per-sub-block list-B
# evaluation vs the HEAD build, interleaved twice), the default bench line, the VBS bench line
# and a rocprofv3 kernel trace of the default bench.  Each step has its own limit; a failure ends the call.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03s4; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" $O/pytest_gpu.log | tail -8; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  timeout -k 10 400 python -u tools/vbs_ab.py tools/_ab/head.so >> $O/vbs_ab.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "vbs_ab rc=$rc"; tail -5 $O/vbs_ab.log; exit $rc; }
done
cat $O/vbs_ab.log
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 600 $O/bench.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --vbs --no-cpu-baseline --no-pcie --no-records > $O/bench_vbs.log 2>&1
rc=$?; echo "bench vbs rc=$rc"; tail -c 600 $O/bench_vbs.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pcie > $O/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
exit $rc
