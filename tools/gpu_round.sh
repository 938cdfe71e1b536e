#!/bin/bash
# One GPU call: the -m gpu suite, the default bench line, then a rocprofv3 kernel trace of a
# short bench.  Each step has its own time limit; a failing step ends the call.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r02}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
      > gpurun_out/pytest_gpu_${TAG}.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" gpurun_out/pytest_gpu_${TAG}.log | tail -8
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench_${TAG}.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/bench_${TAG}.log
[ $rc -ne 0 ] && exit $rc
if [ "${SKIP_PROF:-0}" != 1 ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pcie ${PROF_ARGS} > gpurun_out/prof_${TAG}.log 2>&1
  rc=$?; echo "rocprof rc=$rc"
fi
exit $rc
