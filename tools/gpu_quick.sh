#!/bin/bash
# One GPU call: a -k subset of the -m gpu suite, then bench.py on one config (its own limits).
#   PYK="two_pass or rc2pass" CFG=4k_rc2pass TAG=x bash tools/gpu_quick.sh
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-quick}
if [ -n "$PYK" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "$PYK" --timeout 200 --timeout-method thread \
      -p no:cacheprovider > gpurun_out/pytest_${T}.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_${T}.log; [ $rc -ne 0 ] && exit $rc
fi
for c in ${CFG:-4k}; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-pcie --no-records ${BENCH_ARGS} \
      --detail-out gpurun_out/${T}_$c.json > gpurun_out/bench_${T}_$c.log 2>&1
  rc=$?; echo "bench $c rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_${T}_$c.log; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_${T}_$c.log').read().strip().splitlines()[-1]); print('$c', d['ms_per_step'], d['parity'], d['roofline'])"
done
