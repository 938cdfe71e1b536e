#!/bin/bash
# HBM traffic of every kernel in the bench command (MI355X_MICROARCH.md HBM section):
# FETCH_SIZE and WRITE_SIZE in separate --pmc passes over a short bench run (and one pass of
# SQ instruction counts), then
# tools/traffic_json.py writes profiles/pmc_me_traffic.json (bench.py roofline.traffic).  Run it
# HERE on the merged gpurun_out/traffic: a profiles/ file written on the GPU box does not come back.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/traffic
TAG=${1:-r01}
CFG=${2:-4k}
for c in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"; do
  d=$(echo $c | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/traffic/${TAG}_${CFG}_$d -o run -- \
      python3 bench.py --config $CFG --steps 1 --warmup 1 --kernel-reps 5 --no-cpu-baseline \
      > gpurun_out/traffic/${TAG}_${CFG}_$d.log 2>&1
  rc=$?; echo "pmc $d rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/traffic/${TAG}_${CFG}_$d.log; exit $rc; }
done
exit 0
