#!/bin/bash
# Round-end measurement set: parity suite, 4K bench (with the CPU baseline), rocprof stats of
# the same command, HBM traffic + SQ instruction passes (4K, 1080p), 1080p bench.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_${TAG}.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_${TAG}.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_traffic.sh ${TAG} 4k && python3 tools/traffic_json.py gpurun_out/traffic ${TAG} 4k || exit 1
bash tools/gpu_traffic.sh ${TAG} 1080p && python3 tools/traffic_json.py gpurun_out/traffic ${TAG} 1080p || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_4k_${TAG}.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/bench_4k_${TAG}.log | tail -1 | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_4k_${TAG} -o run -- \
    python3 bench.py --no-cpu-baseline > gpurun_out/prof_4k_${TAG}.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config 1080p --no-cpu-baseline > gpurun_out/bench_1080p_${TAG}.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/bench_1080p_${TAG}.log | tail -1 | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_1080p_${TAG} -o run -- \
    python3 bench.py --config 1080p --no-cpu-baseline > gpurun_out/prof_1080p_${TAG}.log 2>&1 || exit 1
echo done
