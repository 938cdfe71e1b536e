#!/bin/bash
# GPU parity suite (no -x: report every failure); stops the call on a crash code.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider "$@" > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "passed|failed|error|FAILED|ERROR" gpurun_out/pytest_gpu.log | tail -40
exit $rc
