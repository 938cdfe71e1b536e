#!/bin/bash
# me_ab2 (sea variant only) against each A/B library build in tools/_ab/ and the default.
cd "$GRAFT_REPO_ROOT" || exit 1
for lib in "" tools/_ab/*.so; do
  AB_VARIANTS=sea SO_LIB_PATH=$lib timeout -k 10 200 python tools/me_ab2.py > gpurun_out/ab_lib.log 2>&1 || { tail -3 gpurun_out/ab_lib.log; exit 1; }
  echo "lib=${lib:-default}"; grep "pair 1" gpurun_out/ab_lib.log
done
