"""HBM bytes per launch of every so:: kernel from tools/gpu_traffic.sh output.

Usage: python tools/traffic_json.py gpurun_out/traffic <tag> <config>
bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 (KB units; FETCH_SIZE tallies the 128-B
requests of coalesced streaming reads at 64 B on gfx950, MI355X_MICROARCH.md), averaged
over the kernel's dispatches.  Merged into profiles/pmc_me_traffic.json under <config>.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

base, tag, cfg = sys.argv[1], sys.argv[2], sys.argv[3]
vals = defaultdict(dict)
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(base, f"{tag}_{cfg}_{c}", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "so::" in r["Kernel_Name"] and r["Counter_Name"] == c:
                acc[r["Kernel_Name"].replace("void ", "").split("(")[0]].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        vals[k][c] = sum(v) / len(v)
        vals[k][c + "_dispatches"] = len(v)
insts = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(base, f"{tag}_{cfg}_SQ_WAVES", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "so::" in r["Kernel_Name"]:
            insts[r["Kernel_Name"].replace("void ", "").split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
per = {}
for k, v in sorted(vals.items()):
    if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
        per[k] = {"hbm_bytes": 2 * v["FETCH_SIZE"] * 1024 + v["WRITE_SIZE"] * 1024,
                  "fetch_kb": v["FETCH_SIZE"], "write_kb": v["WRITE_SIZE"],
                  "dispatches": v["FETCH_SIZE_dispatches"]}
        if k in insts:
            per[k].update({c.lower(): sum(x) / len(x) for c, x in insts[k].items()})
out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_me_traffic.json")
doc = json.load(open(out)) if os.path.exists(out) else {}
doc["_note"] = ("HBM bytes per launch = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 from separate rocprofv3 --pmc passes "
                "over `bench.py --steps 1 --warmup 1 --kernel-reps 5` (tools/gpu_traffic.sh); sq_* = SQ instruction "
                "counts per launch from one more pass")
doc[cfg] = {"source": f"{base}/{tag}_{cfg}_*", "kernels": per}
json.dump(doc, open(out, "w"), indent=1, sort_keys=True)
for k, v in per.items():
    print(f"{k:40s} {v['hbm_bytes'] / 1e6:9.2f} MB/launch  ({v['dispatches']} dispatches)")
