#!/bin/bash
# 4K GOP throughput of each ME variant (bench.py --me ...), 1 GPU; each run bounded.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-mv}
for me in fme fastpar fast fast_fme; do
  timeout -k 10 300 python bench.py --me $me --steps 2 --warmup 1 --no-cpu-baseline --kernel-reps 3 \
      > gpurun_out/bench_${TAG}_${me}.log 2>&1; rc=$?
  echo "me=$me rc=$rc"; grep -v amdgpu.ids gpurun_out/bench_${TAG}_${me}.log | tail -1 | cut -c1-400
  [ $rc -ne 0 ] && exit $rc
done
exit 0
