"""P-run per-frame time of the default library vs A/B builds (SO_LIB_PATH) or environment
settings, each in a fresh process:
    python tools/ab_runs.py tools/_ab/a.so SO_RUN_PER_CU=2 ...   (one JSON line per variant)"""
import json
import os
import subprocess
import sys

CHILD = r'''
import json, os, sys, time, torch
sys.path.insert(0, ".")
from streamoptima_amd.engine import Engine, alloc_planes
from streamoptima_amd.synth import synth_sequence_torch
sys.path.insert(0, "tools")
from ab_guard import require_ab_build  # noqa: E402  (the child runs from the repo root)
require_ab_build()
dev = torch.device("cuda:0")
out = {}
for h, w in ((2160, 3840), (1088, 1920), (272, 3840)):
    f = 30
    eng = Engine(h, w, 16, 16, os.environ.get("SO_AB_VBS") == "1", 0.015, dev)
    fr = alloc_planes(f, h, w, dev)
    fr.copy_(synth_sequence_torch(f, h, w, seed=0, device=dev, content=os.environ.get("SO_AB_CONTENT", "bench")))
    i0 = eng.encode_i(fr[0], 4)
    outs = [eng.new_symbols(1) for _ in range(f - 1)]
    ts = []
    for _ in range(7):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        eng.encode_p_run([fr[i] for i in range(1, f)], i0.recon, 4, outs)
        torch.cuda.synchronize(); ts.append(time.perf_counter() - t0)
    eng.check_run()
    ts = sorted(ts[1:])
    out[f"{w}x{h}"] = [round(ts[0] / (f - 1) * 1e6, 2), round(ts[len(ts) // 2] / (f - 1) * 1e6, 2)]
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
        print(json.dumps({"lib": lib or "default", "us_per_frame_min_median": json.loads(line[-1]) if line else r.stderr[-500:]}),
              flush=True)


if __name__ == "__main__":
    main()
