"""fast_me mode-0 ME time per P-frame (the serial predictor chain, Encoder.py:462-585) on the
bench's 4K content: the one-wavefront walk (SO_FASTME_SERIAL=1) vs the segment speculation,
and how many segments the in-order check had to redo.  Each variant in a fresh process:
    python tools/fastme_probe.py [SO_FASTME_K=16,SO_FASTME_WARM=16 ...]"""
import json
import os
import subprocess
import sys

CHILD = r'''
import ctypes, json, sys, time, torch
sys.path.insert(0, ".")
from streamoptima_amd import _lib
from streamoptima_amd.engine import Engine, alloc_planes
from streamoptima_amd.synth import synth_sequence_torch
dev = torch.device("cuda:0")
h, w = 2160, 3840
fr = alloc_planes(3, h, w, dev)
fr.copy_(synth_sequence_torch(3, h, w, seed=0, device=dev))
import os
sys.path.insert(0, "tools")
from ab_guard import require_ab_build  # noqa: E402  (the child runs from the repo root)
require_ab_build()
eng = Engine(h, w, 16, 16, os.environ.get("PROBE_VBS") == "1", 0.015, dev, me_mode=_lib.ME_FAST)
i0 = eng.encode_i(fr[0], 4)
p1 = eng.encode_p(fr[1], [i0.recon], 4)
out = eng.new_symbols(1)
ts = []
for _ in range(5):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    eng.encode_p(fr[2], [p1.recon], 4, out=out)
    torch.cuda.synchronize(); ts.append(time.perf_counter() - t0)
n = ctypes.c_int(-1)
lib = _lib.load()
lib.so_debug_fast_chain_fixed(ctypes.byref(n))
ts.sort()
print(json.dumps({"ms_per_p_frame_min_median": [round(ts[0] * 1e3, 3), round(ts[2] * 1e3, 3)],
                  "segments_redone_last": n.value}))
'''


def main():
    for v in ["SO_FASTME_SERIAL=1", ""] + sys.argv[1:]:   # PROBE_VBS=1 in a variant: VBSEnable
        env = dict(os.environ)
        for kv in v.split(","):
            if kv:
                k, val = kv.split("=", 1)
                env[k] = val
        r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        print(json.dumps({"variant": v or "default", **(json.loads(line[-1]) if line else {"err": r.stderr[-600:]})}),
              flush=True)


if __name__ == "__main__":
    main()
