"""Per-implementation ME counter table from tools/gpu_pmc_me.sh output."""
import csv, glob, os, sys
from collections import defaultdict
base, tag = sys.argv[1], sys.argv[2]
for impl in ("sea", "sea2", "sea1", "dense", "wave", "tile", "fast"):
    c = defaultdict(list)
    for f in glob.glob(os.path.join(base, f"{tag}_{impl}_p*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if "me_" in r["Kernel_Name"]:
                c[r["Counter_Name"]].append(float(r["Counter_Value"]))
    a = {k: sum(v) / len(v) for k, v in c.items()}
    if not a:
        continue
    wc = a.get("SQ_WAVE_CYCLES", 1)
    print(f"== {impl}: waves={a.get('SQ_WAVES',0):.0f} valu/wave={a.get('SQ_INSTS_VALU',0)/max(a.get('SQ_WAVES',1),1):.0f} "
          f"lds/wave={a.get('SQ_INSTS_LDS',0)/max(a.get('SQ_WAVES',1),1):.0f} smem/wave={a.get('SQ_INSTS_SMEM',0)/max(a.get('SQ_WAVES',1),1):.0f}")
    for k in sorted(a):
        extra = f"  ({a[k]/wc:.3f} of wave-cycles)" if k.startswith(("SQ_WAIT", "SQ_ACTIVE", "SQ_THREAD")) else ""
        print(f"   {k:28s} {a[k]:.4g}{extra}")
