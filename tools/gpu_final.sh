#!/bin/bash
# The round's final measurements in one GPU call, each step with its own limit:
#   the -m gpu suite; the driver's default bench line; a rocprofv3 kernel trace of the headline
#   workload alone (4K GOP, no records: its p_run_kernel average is the line's launch time) and
#   of each record workload alone (per-config kernel stats for profiles/).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-final}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
      > gpurun_out/pytest_gpu_${T}.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu_${T}.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 600 python -u bench.py --detail-out gpurun_out/${T}_detail.json > gpurun_out/bench_${T}.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -c 1500 gpurun_out/bench_${T}.log; exit $rc; }
for cfg in ${PROF_CFGS:-4k 1080p 4k_vbs 4k_rc2pass 4k_noise}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${T}_$cfg -o run -- \
      python3 bench.py --config $cfg --steps 5 --warmup 1 --no-cpu-baseline --no-pcie --no-records --detail-out '' \
      > gpurun_out/prof_${T}_$cfg.log 2>&1
  rc=$?; echo "rocprof $cfg rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
