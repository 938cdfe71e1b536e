#!/bin/bash
# 2x2-cell SEA for dense-predicted tiles (sea_fine_block): the dense-tile parity tests, the GPU
# suite, then the P-run A/B against the build without it (tools/_ab/nofine.so, -DSO_DENSE_FINE=0)
# on noise, low-texture and benchmark content.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -x -v -m gpu --timeout 200 --timeout-method thread \
    -p no:cacheprovider -k "dense_predicted or noise or lowtex" > gpurun_out/pytest_r04j_dense.log 2>&1
rc=$?; echo "pytest dense rc=$rc"; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/pytest_r04j_dense.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_gpu_r04j.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu_r04j.log; [ $rc -eq 0 ] || exit $rc
for c in noise lowtex bench; do
  SO_AB_CONTENT=$c TAG=r04_fine_$c AB_TIMEOUT=400 ROUNDS=2 VARIANTS="tools/_ab/nofine.so" bash tools/gpu_ab_r04.sh || exit $?
done
