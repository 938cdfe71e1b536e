#!/bin/bash
# Dense tiles over four window copies (copies 1..3 staged into the scratch): the GPU suite on
# the in-tree library, then the P-run A/B against the single-copy build (tools/_ab/one.so,
# -DSO_DENSE_ONE) on noise, low-texture and benchmark content, and VBS on noise.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_gpu_r04i.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_r04i.log; [ $rc -eq 0 ] || exit $rc
for c in noise lowtex bench; do
  SO_AB_CONTENT=$c TAG=r04_dense_$c AB_TIMEOUT=400 ROUNDS=2 VARIANTS="tools/_ab/one.so" bash tools/gpu_ab_r04.sh || exit $?
done
SO_AB_VBS=1 SO_AB_CONTENT=noise TAG=r04_dense_vbs_noise AB_TIMEOUT=400 ROUNDS=2 VARIANTS="tools/_ab/one.so" bash tools/gpu_ab_r04.sh
