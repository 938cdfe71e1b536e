#!/bin/bash
# Whole-GOP A/B of the in-tree library against one variant ($1) by alternating bench.py runs
# (headline config, or --config $CFG), then a rocprofv3 kernel-stats pass of each.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pair
A="--steps 20 --warmup 5 --no-records --no-pcie --no-cpu-baseline ${CFG:+--config $CFG}"
for r in 1 2 3; do
  for v in default "$1"; do
    if [ "$v" = default ]; then env -u SO_LIB_PATH timeout -k 10 300 python bench.py $A > gpurun_out/pair/b.log 2>&1 || exit 1
    else SO_LIB_PATH=$v timeout -k 10 300 python bench.py $A > gpurun_out/pair/b.log 2>&1 || exit 1; fi
    python -c "import json;d=[json.loads(l) for l in open('gpurun_out/pair/b.log') if l.startswith('{')][-1];print('$v', d['ms_per_step'], d['parity']['bit_exact'])"
  done
done | tee gpurun_out/pair/summary.log
for v in default "$1"; do
  n=$(basename $v .so)
  if [ "$v" = default ]; then X=""; else X="$v"; fi
  SO_LIB_PATH=$X timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pair/prof_$n -o run -- \
      python3 bench.py --steps 3 --warmup 1 --no-records --no-pcie --no-cpu-baseline --no-parity ${CFG:+--config $CFG} \
      > gpurun_out/pair/prof_$n.log 2>&1 || exit 1
done
exit 0
