"""Per-kernel SQ counter table from tools/gpu_pmc_gop.sh output (averaged over dispatches)."""
import csv, glob, os, sys
from collections import defaultdict
base, tag = sys.argv[1], sys.argv[2]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(base, f"{tag}_p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "so::" not in k:
            continue
        acc[k.split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in sorted(acc.items()):
    a = {n: sum(v) / len(v) for n, v in c.items()}
    w = max(a.get("SQ_WAVES", 1), 1)
    wc = a.get("SQ_WAVE_CYCLES", 1)
    print(f"== {k}: waves={w:.0f} valu/wave={a.get('SQ_INSTS_VALU', 0) / w:.0f} "
          f"salu/wave={a.get('SQ_INSTS_SALU', 0) / w:.0f} lds/wave={a.get('SQ_INSTS_LDS', 0) / w:.0f} "
          f"vmem/wave={a.get('SQ_INSTS_VMEM', 0) / w:.0f}")
    for n in sorted(a):
        extra = f"  ({a[n] / wc:.3f} of wave-cycles)" if n.startswith(("SQ_WAIT", "SQ_ACTIVE")) else ""
        print(f"   {n:24s} {a[n]:.4g}{extra}")
