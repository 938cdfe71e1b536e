#!/bin/bash
# bench.py --gpus N rehearsal on a one-GPU box: N ranks share cuda:0 (gloo collectives, capped
# persistent grids).  Exercises the rank launch, the p2p hand-off setup + self-check, the timed
# strong-scaling loop and the parity check of configs[3]; the numbers are not a scaling result.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for n in ${NS:-2 4}; do
  timeout -k 10 400 python -u bench.py --gpus $n --share-gpu --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} \
      > gpurun_out/bench_share_$n.log 2>&1
  rc=$?; echo "N=$n rc=$rc"
  grep -o '"value": [0-9.]*\|"n_gpus": [0-9]*\|"bit_exact": [a-z]*\|"parallelism": "[^"]*"\|"ms_per_step": [0-9.]*' gpurun_out/bench_share_$n.log | tr '\n' ' '; echo
  [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_share_$n.log; exit $rc; }
done
exit 0
