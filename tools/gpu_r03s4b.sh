#!/bin/bash
# Kernel trace of the 1080p and 4K single-GOP benches (per-GOP kernel sequence, gaps, I-frame cost).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03s4b; mkdir -p $O
for c in 1080p 4k; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o run -- \
      python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-pcie --no-records --no-content-records \
      > $O/bench_$c.log 2>&1
  rc=$?; echo "$c rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/bench_$c.log; exit $rc; }
done
exit 0
