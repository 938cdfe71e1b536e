"""Summarise tools/gpu_pmc_variants.sh: per variant, the P-run kernel's issue and stall counters
per launch -- VALU instructions, VALU busy, resident waves per SIMD, and where wave-cycles go.

    python tools/pmc_variants.py gpurun_out/<TAG> [variant ...]
Counter units (MI355X_MICROARCH.md): SQ_*_CYCLES / SQ_ACTIVE_INST_* / SQ_WAIT_* in quad-cycles
summed over waves; GRBM_GUI_ACTIVE summed over the 8 XCDs."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

N_SIMD = 1024


def load(d):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("void ", "").split("(")[0]
            if "p_run_kernel" in k:
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v[1:] or v) / len(v[1:] or v) for c, v in cs.items()} for k, cs in acc.items()}


def summary(base, n):
    out = {}
    for p in ("sq1", "sq2"):
        for k, v in load(os.path.join(base, f"{n}_{p}")).items():
            out.setdefault(k, {}).update(v)
    res = {}
    for k, v in out.items():
        cyc = v["GRBM_GUI_ACTIVE"] / 8
        r = {"kernel_cycles": round(cyc), "valu_insts": round(v.get("SQ_INSTS_VALU", 0)),
             "valu_busy": round(4 * v.get("SQ_ACTIVE_INST_VALU", 0) / (cyc * N_SIMD), 4),
             "waves_per_simd": round(4 * v.get("SQ_WAVE_CYCLES", 0) / (cyc * N_SIMD), 2),
             "lds_insts": round(v.get("SQ_INSTS_LDS", 0)), "salu_insts": round(v.get("SQ_INSTS_SALU", 0))}
        wc = v.get("SQ_WAVE_CYCLES")
        if wc and "SQ_WAIT_ANY" in v:
            r.update({"wait_any_frac": round(v["SQ_WAIT_ANY"] / wc, 4),
                      "wait_inst_any_frac": round(v["SQ_WAIT_INST_ANY"] / wc, 4),
                      "active_inst_any_frac": round(v["SQ_ACTIVE_INST_ANY"] / wc, 4),
                      "wait_inst_lds_frac": round(v["SQ_WAIT_INST_LDS"] / wc, 4),
                      "lds_bank_conflict_cycles": round(v.get("SQ_LDS_BANK_CONFLICT", 0)),
                      "vmem_insts": round(v.get("SQ_INSTS_VMEM", 0)), "smem_insts": round(v.get("SQ_INSTS_SMEM", 0))})
        res[k] = r
    return res


if __name__ == "__main__":
    base = sys.argv[1]
    names = sys.argv[2:] or sorted({os.path.basename(p).rsplit("_", 1)[0] for p in glob.glob(os.path.join(base, "*_sq1"))})
    print(json.dumps({n: summary(base, n) for n in names}, indent=1))
