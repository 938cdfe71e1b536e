#!/bin/bash
# The -m gpu suite in one process, with a per-test time limit and a whole-run limit.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-tests}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS} \
    > gpurun_out/pytest_gpu_$T.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR|Error" gpurun_out/pytest_gpu_$T.log | tail -15
exit $rc
