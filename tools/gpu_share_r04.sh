#!/bin/bash
# Multi-rank rehearsal on one GPU (--share-gpu: every rank on cuda:0, gloo, grids capped): the
# bench's N-rank path (frame pipeline at N >= 3, stripes at N = 2) end to end, bit-exact.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for n in ${NS:-2 4}; do
  timeout -k 10 400 python bench.py --gpus $n --share-gpu --steps 2 --warmup 1 ${SHARE_ARGS} > gpurun_out/bench_share_$n.log 2>&1
  rc=$?; echo "share $n rc=$rc"; grep -o '"parallelism": "[^"]*"\|"bit_exact": [a-z]*\|"timeouts": [0-9]*\|"ms_per_step": [0-9.]*' gpurun_out/bench_share_$n.log | head -5
  [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_share_$n.log; exit $rc; }
done
exit 0
