#!/bin/bash
# Round-3 session 2: headline bench (no CPU leg / records) + its rocprof kernel stats, and the
# resident-workgroups-per-CU A/B (tools/ab_runs.py).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03q; mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline --no-records --no-pcie --no-content-records > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids $O/bench.log | tail -1 | cut -c1-400; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 bench.py --no-cpu-baseline --no-records --no-pcie --no-content-records > $O/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/ab_runs.py SO_RUN_PER_CU=1 SO_RUN_PER_CU=2 SO_RUN_PER_CU=3 > $O/ab_percu.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids $O/ab_percu.log
exit $rc
