#!/bin/bash
# Round-3 session 3: the default bench line (as the driver runs it) and the lean bench's rocprof
# kernel stats, after the intra scan and the integer first transform pass.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03z}; mkdir -p $O
timeout -k 10 900 python bench.py > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids $O/bench.log | tail -1 | cut -c1-600; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 bench.py --no-cpu-baseline --no-records --no-pcie --no-content-records > $O/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
