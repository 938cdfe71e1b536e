"""Static VALU census of the persistent run kernel by phase (round 5, VERDICT r04 "Next 3").

Compiles so_me.hip to gfx950 assembly with -DSO_MARKS (a `;SO_MARK name` comment line at each
phase boundary of p_run_kernel's persistent loop, so_me.hip SO_MARK) and attributes every
instruction of the kernel to the last marker above it in layout order.  Prints, per phase, the
static counts of VALU instructions, of them FP64 / v_sad / v_readlane+v_writelane (SGPR spill
traffic through VGPR lanes) / scratch (VGPR spills), and LDS and global memory instructions.

    python tools/isa_census.py [--kernel 'p_run_kernel<8, 0, false, false>'] [-D DEFINE ...]

Static counts are per code path; tools/valu_model.py weights them by how often each phase runs
per block."""
import argparse
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def mangled(kernel: str) -> str:
    m = re.match(r"p_run_kernel<(\d+), (\d+), (true|false), (true|false)(?:, (true|false))?(?:, (true|false))?>",
                 kernel)
    if not m:
        raise SystemExit(f"kernel {kernel!r}: expected p_run_kernel<NW, MODE, VBS, HOOKS, UQP, ZSKIP>")
    b = lambda v: "1" if v == "true" else "0"   # noqa: E731
    return (f"_ZN2so12p_run_kernelILi{m.group(1)}ELi{m.group(2)}ELb{b(m.group(3))}ELb{b(m.group(4))}"
            f"ELb{b(m.group(5) or 'false')}ELb{b(m.group(6) or 'false')}EEEvNS_8PRunArgsEiPKhiiiPKiPjiNS_10PRunStripeEd")


def census(asm: str, fn: str) -> dict:
    lines = asm.split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(fn + ":"))
    end = next(i for i in range(start, len(lines)) if re.match(r"\s+s_endpgm", lines[i]))
    cur = "prologue"
    out = collections.OrderedDict()
    for l in lines[start:end]:
        m = re.search(r";SO_MARK (\w+)", l)
        if m:
            cur = m.group(1)
            out.setdefault(cur, collections.Counter())["copies"] += 1   # unrolled / duplicated markers
            continue
        ins = l.strip().split(" ")[0] if l.startswith("\t") or l.startswith(" ") else ""
        if not ins or ins.startswith((";", ".")):
            continue
        d = out.setdefault(cur, collections.Counter())
        if ins.startswith("v_"):
            d["valu"] += 1
            if re.match(r"v_(fma|add|mul|ldexp|rndne|fract|trig|div|max|min)_f64|v_cvt_.*f64", ins):
                d["fp64"] += 1
            if ins.startswith("v_sad"):
                d["sad"] += 1
            if ins in ("v_readlane_b32", "v_writelane_b32"):
                d["lane_rw"] += 1
            if ins.startswith("v_readfirstlane"):
                d["readfirstlane"] += 1
        elif ins.startswith("s_"):
            d["salu_smem"] += 1
        elif ins.startswith("ds_"):
            d["lds"] += 1
        elif ins.startswith("scratch_"):
            d["scratch"] += 1
        elif ins.startswith(("global_", "buffer_", "flat_")):
            d["vmem"] += 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="p_run_kernel<8, 0, false, false, false, false>")
    ap.add_argument("-D", dest="defines", action="append", default=[])
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as tmp:
        s = os.path.join(tmp, "so_me.s")
        r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                            "-I", os.path.join(ROOT, "include"), "-DSO_MARKS", *[f"-D{d}" for d in a.defines],
                            "--cuda-device-only", "-S", os.path.join(ROOT, "streamoptima_amd/csrc/so_me.hip"), "-o", s],
                           capture_output=True, text=True)
        if r.returncode:
            raise SystemExit(r.stderr[-3000:])
        res = census(open(s).read(), mangled(a.kernel))
    if a.json:
        print(json.dumps({k: dict(v) for k, v in res.items()}))
        return
    cols = ("copies", "valu", "fp64", "sad", "lane_rw", "readfirstlane", "scratch", "lds", "vmem", "salu_smem")
    print(f"{a.kernel}  (static instructions per phase, layout order)")
    print(f"{'phase':16s}" + "".join(f"{c:>14s}" for c in cols))
    tot = collections.Counter()
    for k, v in res.items():
        tot.update(v)
        print(f"{k:16s}" + "".join(f"{v.get(c, 0):14d}" for c in cols))
    print(f"{'TOTAL':16s}" + "".join(f"{tot.get(c, 0):14d}" for c in cols))


if __name__ == "__main__":
    main()
