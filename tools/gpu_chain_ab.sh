#!/bin/bash
# stripe-height chain probe for the default library and each tools/_ab/*.so
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-chainab}
shopt -s nullglob
for lib in "" tools/_ab/*.so; do
  SO_LIB_PATH=$lib timeout -k 10 300 python -u tools/stripe_chain.py ${CHAIN_ARGS} > gpurun_out/chain_$T.log 2>&1
  rc=$?; echo "lib=${lib:-default} rc=$rc"; grep "H=" gpurun_out/chain_$T.log
  [ $rc -ne 0 ] && { tail -5 gpurun_out/chain_$T.log; exit $rc; }
done
exit 0
