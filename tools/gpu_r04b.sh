#!/bin/bash
# Round-4 check: the new GPU tests (waits, residency claims), then the wait-loop A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_waits.py tests/test_gpu_pipeline.py -x -v -m gpu --timeout 120 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r04b.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_r04b.log | tail -8
[ $rc -ne 0 ] && exit $rc
TAG=r04_wait AB_TIMEOUT=900 ROUNDS=4 VARIANTS="tools/_ab/old.so tools/_ab/simple.so tools/_ab/call.so" bash tools/gpu_ab_r04.sh
