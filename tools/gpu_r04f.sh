#!/bin/bash
# The matrix-core forward transform (tools/_ab/mfma.so, -DSO_FWD_MFMA=1): the whole GPU suite
# through that library, then the interleaved P-run A/B against the in-tree library.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
SO_LIB_PATH=tools/_ab/mfma.so timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_mfma.log 2>&1
rc=$?; echo "pytest mfma rc=$rc"; tail -5 gpurun_out/pytest_mfma.log; [ $rc -eq 0 ] || exit $rc
TAG=r04_mfma AB_TIMEOUT=600 ROUNDS=${ROUNDS:-3} VARIANTS="tools/_ab/mfma.so" bash tools/gpu_ab_r04.sh
