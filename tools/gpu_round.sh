#!/bin/bash
# One GPU call: parity suite -> bench (with CPU baseline) -> rocprofv3 kernel trace of a short bench.
# Each step has its own time limit; a crash/timeout code stops the call.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01}
crashed() { [ "$1" -ge 2 ]; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" gpurun_out/pytest_gpu.log | tail -20
  crashed $rc && exit $rc
fi
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench_${TAG}.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_${TAG}.log
[ $rc -ne 0 ] && exit $rc
if [ "${SKIP_PROF:-0}" != 1 ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ${PROF_ARGS} > gpurun_out/prof_${TAG}.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/prof_${TAG}.log
  find gpurun_out/prof_${TAG} -name "*stats*" | head
fi
