#!/bin/bash
# PMC passes (tools/gpu_traffic.sh) for every benchmarked configuration named in $CFGS, so each
# bench record's roofline carries its own VALU busy fraction and HBM traffic, folded on the box
# into gpurun_out/pmc_me_traffic.json (tools/traffic_json.py, starting from the committed file);
# then a rocprofv3 kernel-trace summary of each configuration's short bench.  Only the summaries
# come back (the raw per-dispatch CSVs exceed gpurun's 64 MiB).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-r05}
mkdir -p gpurun_out/traffic gpurun_out/pmc_${TAG}
export PMC_JSON=gpurun_out/pmc_me_traffic.json
cp profiles/pmc_me_traffic.json $PMC_JSON
for cfg in ${CFGS:-4k 1080p 4k_vbs 4k_rc2pass 4k_lowtex 4k_noise}; do
  bash tools/gpu_traffic.sh $TAG $cfg || exit $?
  python tools/traffic_json.py gpurun_out/traffic $TAG $cfg > gpurun_out/pmc_${TAG}/traffic_${cfg}.txt 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/traffic/${TAG}_${cfg}_trace -o run -- \
      python3 bench.py --config $cfg --steps 3 --warmup 1 --kernel-reps 5 --no-cpu-baseline --no-records --no-pcie \
      --no-parity > gpurun_out/pmc_${TAG}/trace_${cfg}.log 2>&1
  rc=$?; echo "trace $cfg rc=$rc"; [ $rc -ne 0 ] && exit $rc
  f=$(find gpurun_out/traffic/${TAG}_${cfg}_trace -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && cp "$f" gpurun_out/pmc_${TAG}/kernel_stats_${cfg}.csv
  rm -rf gpurun_out/traffic/${TAG}_${cfg}_*
done
rm -rf gpurun_out/traffic
exit 0
