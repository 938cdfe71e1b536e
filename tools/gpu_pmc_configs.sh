#!/bin/bash
# PMC passes (tools/gpu_traffic.sh) for every benchmarked configuration named in $CFGS, so each
# bench record's roofline carries its own VALU busy fraction and HBM traffic; then a rocprofv3
# kernel-trace summary of each configuration's short bench (the per-kernel times).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/traffic
TAG=${TAG:-r04}
for cfg in ${CFGS:-4k 1080p 4k_vbs 4k_rc2pass 4k_lowtex 4k_noise}; do
  bash tools/gpu_traffic.sh $TAG $cfg || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/traffic/${TAG}_${cfg}_trace -o run -- \
      python3 bench.py --config $cfg --steps 3 --warmup 1 --kernel-reps 5 --no-cpu-baseline --no-records --no-pcie \
      --no-parity > gpurun_out/traffic/${TAG}_${cfg}_trace.log 2>&1
  rc=$?; echo "trace $cfg rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
