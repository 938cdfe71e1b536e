#!/bin/bash
# bench A/B (default lib vs tools/_ab/*.so) on the headline config, then the stripe-height chain probe.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-ab}
shopt -s nullglob
for lib in "" tools/_ab/*.so; do
  SO_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-pcie --kernel-reps 10 ${BENCH_ARGS} \
      > gpurun_out/ab_$T.log 2>&1 || { tail -5 gpurun_out/ab_$T.log; exit 1; }
  echo "lib=${lib:-default} $(grep -o '"ms_per_step": [0-9.]*\|"per_frame_us": [0-9.]*\|"bit_exact": [a-z]*' gpurun_out/ab_$T.log | tr '\n' ' ')"
done
if [ "${CHAIN:-1}" = 1 ]; then
  timeout -k 10 300 python -u tools/stripe_chain.py ${CHAIN_ARGS} > gpurun_out/chain_$T.log 2>&1
  rc=$?; echo "chain rc=$rc"; grep "H=" gpurun_out/chain_$T.log
  exit $rc
fi
