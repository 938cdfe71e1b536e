#!/bin/bash
# ME A/B only (tools/me_ab.py), then the ME + stripe parity tests.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-ab}
timeout -k 10 300 python tools/me_ab.py > gpurun_out/me_ab_${TAG}.log 2>&1; rc=$?
echo "me_ab rc=$rc"; grep -v amdgpu.ids gpurun_out/me_ab_${TAG}.log | tail -16
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -m pytest tests -q -m gpu -p no:cacheprovider -x > gpurun_out/pytest_gpu_${TAG}.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" gpurun_out/pytest_gpu_${TAG}.log | tail -8
exit $rc
