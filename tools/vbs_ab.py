"""VBSEnable persistent-run A/B: per-frame time of the 4K / 1088p VBS P-run (p_run_kernel<8, 0,
true>) for the product library and the builds named on the command line (SO_LIB_PATH), each in
a fresh process, plus the count of blocks that took the dense search.
    python tools/vbs_ab.py tools/_ab/vbsdense.so"""
import json
import os
import subprocess
import sys

CHILD = r'''
import json, sys, time, torch
sys.path.insert(0, ".")
from streamoptima_amd.engine import Engine, alloc_planes
from streamoptima_amd.synth import synth_sequence_torch
dev = torch.device("cuda:0")
out = {}
for h, w in ((2160, 3840), (1088, 1920)):
    f = 30
    eng = Engine(h, w, 16, 16, True, 0.015, dev)
    fr = alloc_planes(f, h, w, dev)
    fr.copy_(synth_sequence_torch(f, h, w, seed=0, device=dev))
    i0 = eng.encode_i(fr[0], 4)
    outs = [eng.new_symbols(1) for _ in range(f - 1)]
    eng.encode_p_run([fr[i] for i in range(1, f)], i0.recon, 4, outs)
    torch.cuda.synchronize()
    eng.take_fallback_count()
    ts = []
    for _ in range(5):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        eng.encode_p_run([fr[i] for i in range(1, f)], i0.recon, 4, outs)
        torch.cuda.synchronize(); ts.append(time.perf_counter() - t0)
    eng.check_run()
    fb = eng.take_fallback_count() / 5
    ts = sorted(ts)
    out[f"{w}x{h}"] = {"us_per_frame_min_median": [round(ts[0] / (f - 1) * 1e6, 2), round(ts[2] / (f - 1) * 1e6, 2)],
                       "dense_blocks_frac": round(fb / ((f - 1) * eng.nb), 4)}
print(json.dumps(out))
'''


def main():
    for lib in [""] + sys.argv[1:]:
        env = dict(os.environ)
        if lib:
            env["SO_LIB_PATH"] = lib
        r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        print(json.dumps({"lib": lib or "default", "vbs_p_run": json.loads(line[-1]) if line else r.stderr[-800:]}),
              flush=True)


if __name__ == "__main__":
    main()
