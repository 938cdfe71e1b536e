"""Print per-kernel VGPR/SGPR/spill/LDS/occupancy for the gfx950 build (hipcc remarks)."""
import glob, os, re, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
srcs = sys.argv[1:] or sorted(glob.glob(os.path.join(ROOT, "streamoptima_amd/csrc/*.hip")))
for src in srcs:
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                        "-I", os.path.join(ROOT, "include"), *os.environ.get("KR_DEFINES", "").split(), "-c", src, "-o", "/tmp/_kr.o",
                        "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
    cur = None; rows = []
    for line in r.stderr.splitlines():
        m = re.search(r"remark:\s+(.*?): (.*?) \[-Rpass", line)
        if not m: continue
        k, v = m.group(1), m.group(2)
        if k == "Function Name":
            cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}; rows.append(cur)
        elif cur is not None:
            cur[k] = v
    for c in rows:
        print(f"{c['name'][:70]:70s} vgpr={c.get('VGPRs')} agpr={c.get('AGPRs')} sgpr={c.get('TotalSGPRs')} "
              f"vspill={c.get('VGPRs Spill')} scratch={c.get('ScratchSize [bytes/lane]')} "
              f"occ={c.get('Occupancy [waves/SIMD]')} lds={c.get('LDS Size [bytes/block]')}")
