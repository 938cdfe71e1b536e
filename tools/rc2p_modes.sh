#!/bin/bash
# configs[4] (4K ROI + two-pass RC GOP) in its three execution modes, alternating processes:
# the Python per-frame loop (default), the library-enqueued per-frame sequence (SO_RUN_2PASS=1)
# and both passes in one persistent launch (SO_RUN_2PASS=1 + SO_OPT_RUN_2PASS_FUSED); fusedv: the
# fused run through the variant library $VLIB.  MODES picks the modes.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
A="--config 4k_rc2pass --steps 10 --warmup 3 --no-records --no-pcie --no-cpu-baseline"
for r in 1 2; do
  for m in ${MODES:-loop lib fused}; do
    case $m in
      loop) env -u SO_RUN_2PASS timeout -k 10 300 python bench.py $A > gpurun_out/rc.log 2>&1 || exit 1 ;;
      lib) SO_RUN_2PASS=1 timeout -k 10 300 python bench.py $A > gpurun_out/rc.log 2>&1 || exit 1 ;;
      fusedv) SO_LIB_PATH=$VLIB SO_RUN_2PASS=1 timeout -k 10 300 python -c "import sys; sys.argv=['bench.py']+sys.argv[1:]; from streamoptima_amd import _lib; _lib.set_option(_lib.OPT_RUN_2PASS_FUSED, 1); import bench; bench.main(sys.argv[1:])" $A > gpurun_out/rc.log 2>&1 || exit 1 ;;
      fused) SO_RUN_2PASS=1 timeout -k 10 300 python -c "import sys; sys.argv=['bench.py']+sys.argv[1:]; from streamoptima_amd import _lib; _lib.set_option(_lib.OPT_RUN_2PASS_FUSED, 1); import bench; bench.main(sys.argv[1:])" $A > gpurun_out/rc.log 2>&1 || exit 1 ;;
    esac
    python -c "import json;d=[json.loads(l) for l in open('gpurun_out/rc.log') if l.startswith('{')][-1];print('$m', d['ms_per_step'], d['parity']['bit_exact'])"
  done
done | tee gpurun_out/rc2p_modes.log
