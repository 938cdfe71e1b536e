"""Summarise rocprofv3 --pmc passes (tools/gpu_pmc.sh) per kernel.

Usage: python tools/pmc_summary.py gpurun_out/pmc r01 [profiles/r01]
Averages every counter over the dispatches of each kernel, derives the issue metrics, and
computes HBM traffic per launch as the MI355X_MICROARCH.md HBM section prescribes:
FETCH_SIZE and WRITE_SIZE come from separate passes (KB units); FETCH_SIZE reads half the
bytes of wide coalesced reads on gfx950, so bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.
Writes <out>/pmc_summary.json and, for bench.py's roofline.traffic, profiles/pmc_traffic.json.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d):
    rows = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            rows[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return rows


def short(name):
    n = name.replace("void ", "")
    return n.split("(")[0]


def main():
    base, tag = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join("profiles", tag)
    agg = defaultdict(dict)
    for pas in ("sq1", "sq2", "fetch", "write"):
        d = os.path.join(base, f"{tag}_{pas}")
        for k, ctrs in load(d).items():
            if "so::" not in k:
                continue
            for c, v in ctrs.items():
                agg[short(k)][c] = sum(v) / len(v)
    summary = {}
    for k, c in sorted(agg.items()):
        s = dict(c)
        if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
            wc = c["SQ_WAVE_CYCLES"]
            s["valu_active_per_wave"] = c.get("SQ_ACTIVE_INST_VALU", 0) / wc
            s["wait_any_frac"] = c.get("SQ_WAIT_ANY", 0) / wc
            s["wait_inst_any_frac"] = c.get("SQ_WAIT_INST_ANY", 0) / wc
            s["wait_inst_lds_frac"] = c.get("SQ_WAIT_INST_LDS", 0) / wc
        if "SQ_BUSY_CYCLES" in c and c.get("SQ_WAVES"):
            s["valu_instr_per_wave"] = c.get("SQ_INSTS_VALU", 0) / c["SQ_WAVES"]
        if "FETCH_SIZE" in c:
            s["hbm_bytes"] = 2 * c["FETCH_SIZE"] * 1024 + c.get("WRITE_SIZE", 0) * 1024
        summary[k] = s
    os.makedirs(out, exist_ok=True)
    json.dump(summary, open(os.path.join(out, "pmc_summary.json"), "w"), indent=1, sort_keys=True)
    for k, s in summary.items():
        keys = ("SQ_WAVES", "SQ_INSTS_VALU", "valu_instr_per_wave", "valu_active_per_wave", "wait_any_frac",
                "wait_inst_any_frac", "wait_inst_lds_frac", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE",
                "FETCH_SIZE", "WRITE_SIZE", "hbm_bytes", "GRBM_GUI_ACTIVE")
        print(k)
        print("   " + "  ".join(f"{x}={s[x]:.4g}" for x in keys if x in s))
    traffic = {}
    for k, s in summary.items():
        if "hbm_bytes" in s:
            traffic[k] = s["hbm_bytes"]
    tp = os.path.join("profiles", "pmc_traffic.json")
    json.dump({"source": f"{base}/{tag}_fetch+write (tools/gpu_pmc.sh), bytes per launch = 2*FETCH_SIZE*1024 + "
                         "WRITE_SIZE*1024 (MI355X_MICROARCH.md HBM: FETCH_SIZE halves wide reads on gfx950)",
               "workload": "4K P-frame (tools/frame_one.py, VBS off)", "bytes_per_launch": traffic},
              open(tp, "w"), indent=1)


main()
