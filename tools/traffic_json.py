"""HBM bytes and VALU issue counters per launch of every so:: kernel from tools/gpu_traffic.sh.

Usage: python tools/traffic_json.py gpurun_out/traffic <tag> <config>
  * FETCH_SIZE is corrected by the factor the calibration microbenchmark measured for the
    4-B-per-lane coalesced reads the encoder's staging uses (tools/ubench_fetch.cpp: bytes
    read / FETCH_SIZE bytes); the guide's x2 is the 16-B-per-lane value, reported beside it.
  * hbm_bytes = calib_b32 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024, averaged over dispatches.
  * SQ counters per launch (sq_active_inst_valu in quad-cycles summed over waves,
    grbm_gui_active summed over the 8 XCDs).
Merged into profiles/pmc_me_traffic.json under <config>.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

base, tag, cfg = sys.argv[1], sys.argv[2], sys.argv[3]


def rows(d):
    for f in glob.glob(os.path.join(base, d, "**", "*counter_collection.csv"), recursive=True):
        yield from csv.DictReader(open(f))


def kname(r):
    return r["Kernel_Name"].replace("void ", "").split("(")[0]


calib = {}
acc = defaultdict(list)
for r in rows(f"{tag}_calib"):
    if r["Counter_Name"] == "FETCH_SIZE":
        acc[kname(r)].append(float(r["Counter_Value"]))
read_bytes = 256 << 20
for k, v in acc.items():
    v = v[1:] or v          # the first dispatch can be cold
    calib[k] = read_bytes / (sum(v) / len(v) * 1024)
fac32 = calib.get("read_b32", 2.0)
vals = defaultdict(dict)
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    acc = defaultdict(list)
    for r in rows(f"{tag}_{cfg}_{c}"):
        if "so::" in r["Kernel_Name"] and r["Counter_Name"] == c:
            acc[kname(r)].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        vals[k][c] = sum(v) / len(v)
        vals[k][c + "_dispatches"] = len(v)
insts = defaultdict(lambda: defaultdict(list))
for r in rows(f"{tag}_{cfg}_SQ_WAVES"):
    if "so::" in r["Kernel_Name"]:
        insts[kname(r)][r["Counter_Name"]].append(float(r["Counter_Value"]))
per = {}
for k, v in sorted(vals.items()):
    if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
        per[k] = {"hbm_bytes": fac32 * v["FETCH_SIZE"] * 1024 + v["WRITE_SIZE"] * 1024,
                  "hbm_bytes_fetch_x2": 2 * v["FETCH_SIZE"] * 1024 + v["WRITE_SIZE"] * 1024,
                  "fetch_kb": v["FETCH_SIZE"], "write_kb": v["WRITE_SIZE"],
                  "dispatches": v["FETCH_SIZE_dispatches"]}
        if k in insts:
            per[k].update({c.lower(): sum(x) / len(x) for c, x in insts[k].items()})
if not per:   # no counter CSVs for this tag (e.g. the GPU call never ran): keep the committed file
    sys.exit(f"no FETCH_SIZE / WRITE_SIZE rows under {base}/{tag}_{cfg}_*: nothing written")
if not calib:
    sys.exit(f"no calibration rows under {base}/{tag}_calib: nothing written")
out = os.environ.get("PMC_JSON") or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                 "profiles", "pmc_me_traffic.json")
doc = json.load(open(out)) if os.path.exists(out) else {}
doc["_note"] = ("per launch: hbm_bytes = calib_b32 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 from separate rocprofv3 "
                "--pmc passes over `bench.py --steps 1 --warmup 1 --kernel-reps 5` (tools/gpu_traffic.sh); calib = "
                "bytes read / FETCH_SIZE bytes measured by tools/ubench_fetch.cpp; sq_* / grbm_* = SQ issue counters "
                "per launch from one more pass")
doc["_fetch_calibration"] = {"bytes_over_fetch_size": calib, "source": f"{base}/{tag}_calib"}
keep = {k: v for k, v in doc.get(cfg, {}).items() if k not in ("source", "kernels")}   # e.g. phase splits
doc[cfg] = {"source": f"{base}/{tag}_{cfg}_*", "kernels": per, **keep}
json.dump(doc, open(out, "w"), indent=1, sort_keys=True)
print("calibration", calib)
for k, v in per.items():
    print(f"{k:40s} {v['hbm_bytes'] / 1e6:9.2f} MB/launch  ({v['dispatches']} dispatches)")
