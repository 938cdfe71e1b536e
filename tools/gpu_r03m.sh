#!/bin/bash
# PMC counters for the current build (4K bench), the pipeline GPU tests, the 3-rank shared-GPU
# configs[4] bench on the frame pipeline (pass-2 lag cap).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03m; mkdir -p $O
bash tools/gpu_traffic.sh r03m 4k || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py -x -q -m gpu --timeout 200 --timeout-method thread \
    -p no:cacheprovider > $O/pytest_pipeline.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_pipeline.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u bench.py --gpus 3 --share-gpu --config 4k_rc2pass --steps 5 --warmup 1 > $O/bench_share_rc2pass_3.log 2>&1
rc=$?; echo "share rc=$rc"; tail -c 400 $O/bench_share_rc2pass_3.log
exit $rc
