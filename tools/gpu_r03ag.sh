#!/bin/bash
# Round-3 final measurements: PMC traffic / issue passes (4K, 1080p), the default bench line,
# the VBS bench line, and the lean bench's rocprof kernel stats.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03ag; mkdir -p $O
tools/gpu_traffic.sh r03ag 4k > $O/traffic_4k.log 2>&1 || { cat $O/traffic_4k.log; exit 1; }
tools/gpu_traffic.sh r03ag 1080p > $O/traffic_1080p.log 2>&1 || { cat $O/traffic_1080p.log; exit 1; }
echo traffic ok
timeout -k 10 900 python bench.py > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids $O/bench.log | tail -1 | cut -c1-300; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --vbs --no-cpu-baseline --no-records --no-pcie --no-content-records > $O/bench_vbs.log 2>&1
rc=$?; echo "bench vbs rc=$rc"; grep -v amdgpu.ids $O/bench_vbs.log | tail -1 | cut -c1-300; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 bench.py --no-cpu-baseline --no-records --no-pcie --no-content-records > $O/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
