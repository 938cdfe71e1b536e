"""Stall accounting per launch of the persistent run kernels from tools/gpu_stall_pmc.sh.

Usage: python tools/stall_summary.py gpurun_out/stall <tag> <config> [out.json]

Per kernel (so::p_run_kernel<...>), averaged over its dispatches:
  * the disjoint split of wave-cycles (MI355X_MICROARCH.md, rocprofv3 PMC slots):
    SQ_WAIT_ANY (parked on s_waitcnt / barrier) + SQ_WAIT_INST_ANY (ready, not issued) +
    SQ_ACTIVE_INST_ANY (issuing) ~= SQ_WAVE_CYCLES, each as a fraction of SQ_WAVE_CYCLES;
  * SQ_WAIT_INST_LDS (the LDS part of the issue stalls), LDS bank-conflict cycles against all
    LDS-array cycles;
  * per-type issue cycles (VALU / LDS / SALU+SMEM / VMEM / branch) as fractions of the SIMD
    cycles (4 * quad-cycles / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)): VALU busy is the first;
  * waves resident per SIMD, VMEM read / write and SMEM instructions per launch.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

N_SIMD = 1024


def rows(base, d):
    for f in glob.glob(os.path.join(base, d, "**", "*counter_collection.csv"), recursive=True):
        yield from csv.DictReader(open(f))


def kname(r):
    return r["Kernel_Name"].replace("void ", "").split("(")[0]


def collect(base, tag, cfg):
    acc = defaultdict(lambda: defaultdict(list))
    for grp in ("wait", "issue"):
        for r in rows(base, f"{tag}_{cfg}_{grp}"):
            if "p_run_kernel" in r["Kernel_Name"]:
                acc[kname(r)][(grp, r["Counter_Name"])].append(float(r["Counter_Value"]))
    out = {}
    for k, d in acc.items():
        v = {key: sum(x) / len(x) for key, x in d.items()}
        g = lambda grp, c: v.get((grp, c))   # noqa: E731
        wc = g("wait", "SQ_WAVE_CYCLES")
        if not wc:
            continue
        cyc_w = g("wait", "GRBM_GUI_ACTIVE") / 8
        cyc_i = g("issue", "GRBM_GUI_ACTIVE") / 8 if g("issue", "GRBM_GUI_ACTIVE") else None
        simd = lambda q, cyc: round(4 * q / (cyc * N_SIMD), 4) if (q is not None and cyc) else None   # noqa: E731
        rec = {
            "dispatches": len(d[("wait", "SQ_WAVE_CYCLES")]),
            "waves_per_simd": round(4 * wc / (cyc_w * N_SIMD), 3),
            "wave_cycles_split": {
                "parked_wait_any": round(g("wait", "SQ_WAIT_ANY") / wc, 4),
                "issue_stall_wait_inst_any": round(g("wait", "SQ_WAIT_INST_ANY") / wc, 4),
                "issuing_active_inst_any": round(g("wait", "SQ_ACTIVE_INST_ANY") / wc, 4),
                "sum": round((g("wait", "SQ_WAIT_ANY") + g("wait", "SQ_WAIT_INST_ANY") +
                              g("wait", "SQ_ACTIVE_INST_ANY")) / wc, 4),
                "of_which_lds_issue_stall": round(g("wait", "SQ_WAIT_INST_LDS") / wc, 4)},
            "lds": {"bank_conflict_cycles_over_lds_cycles":
                    round(g("wait", "SQ_LDS_BANK_CONFLICT") / g("wait", "SQ_LDS_IDX_ACTIVE"), 4)
                    if g("wait", "SQ_LDS_IDX_ACTIVE") else None},
            "simd_busy": {t: simd(g("issue", f"SQ_ACTIVE_INST_{t.upper()}"), cyc_i)
                          for t in ("valu", "lds", "sca", "vmem", "misc")},
            "per_launch": {"vmem_rd_insts": g("issue", "SQ_INSTS_VMEM_RD"), "vmem_wr_insts": g("issue", "SQ_INSTS_VMEM_WR"),
                           "smem_insts": g("issue", "SQ_INSTS_SMEM"), "kernel_cycles_per_xcd": round(cyc_w)},
        }
        out[k] = rec
    return out


def main():
    base, tag, cfg = sys.argv[1], sys.argv[2], sys.argv[3]
    res = collect(base, tag, cfg)
    if not res:
        sys.exit(f"no p_run_kernel rows under {base}/{tag}_{cfg}_*")
    dst = sys.argv[4] if len(sys.argv) > 4 else None
    doc = {"config": cfg, "source": f"{base}/{tag}_{cfg}_{{wait,issue}} (tools/gpu_stall_pmc.sh)",
           "note": __doc__.split("\n\n")[1].strip(), "kernels": res}
    if dst:
        json.dump(doc, open(dst, "w"), indent=1)
    print(json.dumps(doc["kernels"], indent=1))


if __name__ == "__main__":
    main()
