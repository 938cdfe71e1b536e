#!/bin/bash
# One GPU call: ME A/B (tile vs round-1 kernel, identical outputs) -> parity suite -> bench
# (+ PCIe-inclusive rate, CPU baseline) -> rocprofv3 kernel stats of a short bench.
# Every GPU step has its own time limit; any failure ends the call.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r01}
timeout -k 10 300 python tools/me_ab.py > gpurun_out/me_ab_${TAG}.log 2>&1; rc=$?
echo "me_ab rc=$rc"; grep -v amdgpu.ids gpurun_out/me_ab_${TAG}.log | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu_${TAG}.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" gpurun_out/pytest_gpu_${TAG}.log | tail -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --pcie > gpurun_out/bench_${TAG}.log 2>&1; rc=$?
echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench_${TAG}.log | tail -2
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_${TAG}.log 2>&1; rc=$?
echo "rocprof rc=$rc"; grep -v amdgpu.ids gpurun_out/prof_${TAG}.log | tail -1
exit $rc
