"""I-frame encode time (intra_tq + intra_recon_seq) at 4K and 1088p, default library vs A/B
builds / environment settings, each in a fresh process:  python tools/intra_ab.py tools/_ab/x.so"""
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
    eng = Engine(h, w, 16, 16, False, 0.015, dev)
    fr = alloc_planes(1, h, w, dev)
    fr.copy_(synth_sequence_torch(1, h, w, seed=0, device=dev))
    s = eng.encode_i(fr[0], 4)
    ts = []
    for _ in range(20):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        eng.encode_i(fr[0], 4, out=s)
        torch.cuda.synchronize(); ts.append(time.perf_counter() - t0)
    ts = sorted(ts[2:])
    out[f"{w}x{h}"] = [round(ts[0] * 1e6, 1), round(ts[len(ts) // 2] * 1e6, 1)]
print(json.dumps(out))
'''


def main():
    for lib in [""] + sys.argv[1:]:
        env = dict(os.environ)
        if "=" in lib:
            k, v = lib.split("=", 1)
            env[k] = v
        elif lib:
            env["SO_LIB_PATH"] = lib
        r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        print(json.dumps({"lib": lib or "default", "i_frame_us_min_median": json.loads(line[-1]) if line else r.stderr[-400:]}),
              flush=True)


if __name__ == "__main__":
    main()
