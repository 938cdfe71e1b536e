#!/bin/bash
# Round-3 validation: the -m gpu suite, the default bench line, a rocprofv3 kernel trace of a
# short bench, the VBS variants' bench lines and the two-pass frame-pipeline lag probe.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03k; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" $O/pytest.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 600 $O/bench.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pcie --no-records > $O/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
for c in 4k_vbs 1080p_vbs; do
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-pcie > $O/bench_$c.log 2>&1
  rc=$?; echo "bench $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python -u tools/fpipe2p_probe.py > $O/fpipe2p.log 2>&1
rc=$?; echo "probe rc=$rc"; tail -2 $O/fpipe2p.log
exit $rc
