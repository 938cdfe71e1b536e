#!/bin/bash
# Intra recon on DPP rotations: GPU suite (parity incl. the 4K digests), then bench + rocprof.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03r}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 bench.py --no-cpu-baseline --no-records --no-pcie --no-content-records > $O/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; grep -v amdgpu.ids $O/prof.log | tail -1 | cut -c1-300; [ $rc -ne 0 ] && exit $rc
exit 0
