#!/bin/bash
# Interleaved P-run A/B of the in-tree library against the tools/_ab/*.so variants named in $VARIANTS.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 ${AB_TIMEOUT:-900} python -u tools/ab_interleave.py --rounds ${ROUNDS:-3} default ${VARIANTS} > gpurun_out/ab_${TAG:-r04}.log 2>&1
rc=$?; grep summary gpurun_out/ab_${TAG:-r04}.log; exit $rc
