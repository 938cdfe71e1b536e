#!/bin/bash
# Round 2, first GPU call: parity suite (incl. the benchmarked workloads), the bench line,
# the acquire-fence A/B, the stripe-height chain probe, and a rocprofv3 kernel trace.
# Every GPU step has its own limit; any failure ends the call.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r02a}
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_gpu_$T.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" gpurun_out/pytest_gpu_$T.log | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$T.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench_$T.log
[ $rc -ne 0 ] && exit $rc
for lib in "" tools/_ab/noacq.so; do
  SO_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-records --no-pcie --kernel-reps 10 \
      > gpurun_out/ab_$T.log 2>&1 || { tail -5 gpurun_out/ab_$T.log; exit 1; }
  echo "lib=${lib:-default} $(grep -o '"ms_per_step": [0-9.]*\|"per_frame_us": [0-9.]*\|"bit_exact": [a-z]*' gpurun_out/ab_$T.log | tr '\n' ' ')"
done
timeout -k 10 300 python -u tools/stripe_chain.py > gpurun_out/chain_$T.log 2>&1
rc=$?; echo "chain rc=$rc"; cat gpurun_out/chain_$T.log | tail -6
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$T -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pcie > gpurun_out/prof_$T.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -c 600 gpurun_out/prof_$T.log
exit $rc
