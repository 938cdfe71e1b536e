#!/bin/bash
# GPU parity tests selected by -k (all when empty), each test bounded by --timeout.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-t}
K=${2:-}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
    ${K:+-k "$K"} > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "passed|failed|FAILED|ERROR|Error" gpurun_out/pytest_${TAG}.log | tail -30
exit $rc
