#!/bin/bash
# bench (+CPU baseline) -> rocprofv3 kernel stats of the same command shape -> PMC traffic passes.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r01}
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench_${TAG}.log 2>&1; rc=$?
echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench_${TAG}.log | tail -2
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- \
    python3 bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/prof_${TAG}.log 2>&1; rc=$?
echo "rocprof rc=$rc"; grep -v amdgpu.ids gpurun_out/prof_${TAG}.log | tail -1
[ $rc -ne 0 ] && exit $rc
if [ "${TRAFFIC:-1}" = 1 ]; then bash tools/gpu_traffic.sh ${TAG} 4k || exit $?; fi
exit 0
