#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python tools/me_ab.py > gpurun_out/me_ab.log 2>&1; rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids gpurun_out/me_ab.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -m pytest tests -q -m gpu -p no:cacheprovider -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/pytest_gpu.log | tail
