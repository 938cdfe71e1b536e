#!/bin/bash
# One GPU call: the pack / host-stream GPU tests, then BASELINE.md section 4's region per
# upload granularity and P-run chunk (tools/s4_timeline.py), and one traced timeline.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-s4v}
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "pack or host_stream or zero_skip" --timeout 200 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_${T}.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_${T}.log; [ $rc -ne 0 ] && exit $rc
# VARIANTS: comma-separated "chunk upload" pairs
IFS=, read -ra VS <<< "${VARIANTS:-2 frame,2 chunk,3 chunk,1 chunk}"
for v in "${VS[@]}"; do
  set -- $v
  timeout -k 10 120 python -u tools/s4_timeline.py --chunk $1 --upload $2 --reps 12 --quiet >> gpurun_out/s4v_${T}.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "variant $v rc=$rc"; tail -5 gpurun_out/s4v_${T}.log; exit $rc; }
done
grep wall_ms_min gpurun_out/s4v_${T}.log
timeout -k 10 120 python -u tools/s4_timeline.py --reps 3 > gpurun_out/s4_timeline_${T}.log 2>&1
echo "timeline rc=$?"
