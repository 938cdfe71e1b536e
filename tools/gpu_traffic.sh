#!/bin/bash
# PMC passes over a short bench run (MI355X_MICROARCH.md HBM / rocprofv3 section: one counter
# group per pass): FETCH_SIZE, WRITE_SIZE, and the SQ issue counters (VALU busy), plus the
# FETCH_SIZE calibration microbenchmark (tools/ubench_fetch.cpp: 4-B and 16-B coalesced reads
# of a known byte count).  tools/traffic_json.py then writes profiles/pmc_me_traffic.json
# (bench.py roofline.traffic / roofline.valu) -- run it HERE on the merged gpurun_out/traffic.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/traffic
TAG=${1:-r02}
CFG=${2:-4k}
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for c in FETCH_SIZE WRITE_SIZE "$SQ"; do
  d=$(echo $c | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/traffic/${TAG}_${CFG}_$d -o run -- \
      python3 bench.py --config $CFG --steps 1 --warmup 1 --kernel-reps 5 --no-cpu-baseline --no-records --no-pcie \
      --no-parity > gpurun_out/traffic/${TAG}_${CFG}_$d.log 2>&1
  rc=$?; echo "pmc $d rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/traffic/${TAG}_${CFG}_$d.log; exit $rc; }
done
if [ -x tools/ubench_fetch ]; then
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/traffic/${TAG}_calib -o run -- \
      ./tools/ubench_fetch > gpurun_out/traffic/${TAG}_calib.log 2>&1
  rc=$?; echo "calib rc=$rc"; [ $rc -ne 0 ] && exit $rc
fi
exit 0
