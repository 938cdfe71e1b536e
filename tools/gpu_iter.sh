#!/bin/bash
# Iteration call: GPU parity suite -> bench (no CPU baseline) -> rocprofv3 kernel stats of the
# same bench.  Every GPU step has its own time limit; any failure ends the call.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-it}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -q -x -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
      > gpurun_out/pytest_${TAG}.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" gpurun_out/pytest_${TAG}.log | tail -10
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench_${TAG}.log 2>&1; rc=$?
echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench_${TAG}.log | tail -1
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- \
    python3 bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/prof_${TAG}.log 2>&1; rc=$?
echo "rocprof rc=$rc"
python3 - "$TAG" <<'PY'
import csv, glob, sys
for f in glob.glob(f"gpurun_out/prof_{sys.argv[1]}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "so::" in r["Name"]:
            print(f'{float(r["AverageNs"])/1e3:9.2f} us x{r["Calls"]:>4}  {r["Name"].split("(")[0][:70]}')
PY
exit $rc
