#!/bin/bash
# Round-3 checks: the multi-rank RC / ROI paths (frame pipeline two-pass, RC stripes over two
# processes), then shared-GPU rehearsals of the N-rank bench on configs[4] and the variant benches.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_large.py -x -q -m gpu --timeout 300 \
    --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" $O/pytest.log | tail -8; [ $rc -ne 0 ] && exit $rc
for n in 2 3; do
  timeout -k 10 300 python -u bench.py --gpus $n --share-gpu --config 4k_rc2pass --steps 3 --warmup 1 \
      > $O/bench_share_rc2pass_$n.log 2>&1
  rc=$?; echo "share $n rc=$rc"; tail -c 700 $O/bench_share_rc2pass_$n.log; [ $rc -ne 0 ] && exit $rc
done
for a in "--vbs" "--config 1080p --me fme" "--config 1080p --me fast" "--config 1080p --me fastpar" "--config 1080p --vbs"; do
  t=$(echo $a | tr -d ' -')
  timeout -k 10 300 python -u bench.py $a --steps 5 --warmup 2 --no-cpu-baseline --no-pcie > $O/bench_$t.log 2>&1
  rc=$?; echo "bench $a rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"bit_exact": [a-z]*' $O/bench_$t.log | head -4 | tr '\n' ' '; echo
  [ $rc -ne 0 ] && exit $rc
done
exit 0
