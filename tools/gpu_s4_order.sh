#!/bin/bash
# BASELINE.md section 4's region measured first (default) and after the records (--pcie-last):
# the two must agree once the region's streams own their hardware queues (hwqueue.py).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-s4}
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "pack or host or stream" --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/pytest_${T}.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_${T}.log; [ $rc -ne 0 ] && exit $rc
for order in first last; do
  extra=""; [ $order = last ] && extra="--pcie-last"
  timeout -k 10 400 python -u bench.py --no-cpu-baseline $extra --detail-out gpurun_out/${T}_$order.json \
      > gpurun_out/bench_${T}_$order.log 2>&1
  rc=$?; echo "bench $order rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_${T}_$order.log; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_${T}_$order.log').read().strip().splitlines()[-1]); print('$order', d['ms_per_step'], d.get('section4_region'))"
done
