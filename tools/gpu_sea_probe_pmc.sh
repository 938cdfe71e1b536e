#!/bin/bash
# VALU / SALU / LDS instruction counts of me_sea2_kernel truncated after each phase
# (SO_SEA_PROBE: 1 staging + byte sums, 2 + bounds and U, 4 + survivor masks (and the dense
# fallback), 3 everything but the fallback, 0 full), on the GOP's real reference.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/seaprobe
mkdir -p $OUT
for pr in 0 1 2 4 3; do
  SO_SEA_PROBE=$pr ME_N=3 timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
      --output-format csv -d $OUT/p$pr -o run -- python3 tools/me_one.py > $OUT/p$pr.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "probe $pr rc=$rc"; tail -3 $OUT/p$pr.log; exit $rc; }
  python3 - $OUT/p$pr $pr <<'PY'
import csv, glob, sys
from collections import defaultdict
c = defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "me_sea2" in r["Kernel_Name"]:
            c[r["Counter_Name"]].append(float(r["Counter_Value"]))
a = {k: sum(v) / len(v) for k, v in c.items()}
w = a.get("SQ_WAVES", 1)
print(f"probe {sys.argv[2]}: waves {w:.0f} valu/wave {a.get('SQ_INSTS_VALU',0)/w:.0f} salu/wave {a.get('SQ_INSTS_SALU',0)/w:.0f} lds/wave {a.get('SQ_INSTS_LDS',0)/w:.0f}")
PY
done
