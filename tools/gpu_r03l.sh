#!/bin/bash
# Two-pass frame pipeline, in-process ranks at half capacity: GOP time per pass-2 lag.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03l; mkdir -p $O
timeout -k 10 300 python -u tools/fpipe2p_probe.py --worlds 2,3 --lags 26,16,12,8,5,3 --reps 4 --keep-going > $O/fp_half.log 2>&1
rc=$?; echo "rc=$rc"; grep -v amdgpu.ids $O/fp_half.log | tail -1
[ $rc -ne 0 ] && exit $rc
# one-pass frame pipeline, 3 ranks at exactly the chip's resident capacity (768 // 3 each)
timeout -k 10 200 python -u tools/fpipe_probe.py --worlds 3 --frames 30 > $O/fp_onepass_full.log 2>&1
rc=$?; echo "onepass rc=$rc"; grep -v amdgpu.ids $O/fp_onepass_full.log | tail -2
exit $rc
