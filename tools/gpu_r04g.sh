#!/bin/bash
# fwd_mfma: the certificate's flag rate per content, then the P-run A/B against the never- and
# always-flagged timing builds (what the flagged blocks and the matrix-core phase each cost).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
SO_LIB_PATH=tools/_ab/mfmacnt.so timeout -k 10 300 python -u tools/fwd_flag_rate.py > gpurun_out/fwd_flags.log 2>&1
rc=$?; cat gpurun_out/fwd_flags.log | tail -3; [ $rc -eq 0 ] || exit $rc
TAG=r04_mfma2 AB_TIMEOUT=700 ROUNDS=2 VARIANTS="tools/_ab/mfma.so tools/_ab/noflag.so tools/_ab/allflag.so" bash tools/gpu_ab_r04.sh
