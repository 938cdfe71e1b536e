#!/bin/bash
# A/B of the window rows by sc1 loads without the agent acquire (tools/_ab/sc1.so), then the
# benchmarked-GOP digests through that library.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r04_sc1 AB_TIMEOUT=600 ROUNDS=4 VARIANTS="tools/_ab/sc1.so" bash tools/gpu_ab_r04.sh || exit $?
SO_LIB_PATH=tools/_ab/sc1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py -x -q -m gpu --timeout 200 \
    --timeout-method thread -p no:cacheprovider -k "benchmarked or interleaved" > gpurun_out/pytest_sc1.log 2>&1
rc=$?; echo "pytest sc1 rc=$rc"; tail -3 gpurun_out/pytest_sc1.log; exit $rc
