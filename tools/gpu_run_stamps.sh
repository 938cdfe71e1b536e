#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
SO_LIB_PATH=tools/_ab/stamps.so timeout -k 10 300 python -u tools/run_stamps.py ${STAMP_ARGS} > gpurun_out/run_stamps_${TAG:-x}.log 2>&1
rc=$?; grep "H=" gpurun_out/run_stamps_${TAG:-x}.log; [ $rc -ne 0 ] && tail -5 gpurun_out/run_stamps_${TAG:-x}.log
exit $rc
