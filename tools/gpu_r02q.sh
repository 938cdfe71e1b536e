#!/bin/bash
# Round-2 check: the -m gpu suite, the 2-rank shared-GPU bench (frame pipeline), and a kernel
# trace of the frame-pipeline probe (p_run_kernel<8, 2, 128> next to the one-rank kernel).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_gpu_r02q.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" gpurun_out/pytest_gpu_r02q.log | tail -5
[ $rc -ne 0 ] && exit $rc
NS=2 bash tools/gpu_bench_share.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fpipe -o run -- \
    python3 tools/fpipe_probe.py --worlds 2 > gpurun_out/prof_fpipe.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
