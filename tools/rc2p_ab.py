"""Per-GOP time of the configs[4] workload (4K ROI + two-pass RC) under environment
variants (SO_P2LAG=..., SO_PIPELINE=0), each in a fresh process:
    python tools/rc2p_ab.py SO_P2LAG=1 SO_P2LAG=68 SO_PIPELINE=0"""
import json
import os
import subprocess
import sys

CHILD = r'''
import json, sys, time, torch
sys.path.insert(0, ".")
from bench import build_codec, make_frames, parse
from streamoptima_amd.workloads import WORKLOADS
dev = torch.device("cuda:0")
cfg = dict(WORKLOADS["4k_rc2pass"])
codec = build_codec(cfg, parse([]), dev)
fr = make_frames(cfg, dev, cfg["seed"])
ts = []
for _ in range(6):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    codec.encode_device(fr, cfg["intra_dur"], check=False)
    torch.cuda.synchronize(); ts.append(time.perf_counter() - t0)
codec.engine().check_run()
ts = sorted(ts[1:])
print(json.dumps({"ms_per_gop_min_median": [round(ts[0] * 1e3, 3), round(ts[len(ts) // 2] * 1e3, 3)]}))
'''


def main():
    for v in [""] + sys.argv[1:]:
        env = dict(os.environ)
        if v:
            k, val = v.split("=", 1)
            env[k] = val
        r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        print(json.dumps({"variant": v or "default", **(json.loads(line[-1]) if line else {"err": r.stderr[-400:]})}),
              flush=True)


if __name__ == "__main__":
    main()
