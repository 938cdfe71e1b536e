"""PCIe-inclusive GOP time of hoststream.HostStreamEncoder per P-run chunk size (4K x 30).
    python tools/pcie_sweep.py [--chunks 2,3,4,6,10]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", default="2,3,4,6,10,29")
    ap.add_argument("--reps", type=int, default=8)
    a = ap.parse_args()
    from streamoptima_amd.Encoder import Y_Video_codec
    from streamoptima_amd.engine import alloc_planes
    from streamoptima_amd.hoststream import HostStreamEncoder
    from streamoptima_amd.synth import synth_sequence_torch
    dev = torch.device("cuda:0")
    h, w, f = 2160, 3840, 30
    c = Y_Video_codec(h, w, f, 16, 16, 4, f, 0, 0.015, False, device=dev)
    fr = alloc_planes(f, h, w, dev)
    fr.copy_(synth_sequence_torch(f, h, w, seed=0, device=dev))
    host = fr.cpu().pin_memory()
    t0 = time.perf_counter()
    torch.cuda.synchronize()
    h2d = torch.empty_like(fr)
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        h2d.copy_(host, non_blocking=True)
        torch.cuda.synchronize()
        up = time.perf_counter() - t0
    out = {"h2d_only_ms": round(up * 1e3, 3), "h2d_gbs": round(host.numel() / up / 1e9, 2)}
    for ch in [int(x) for x in a.chunks.split(",")]:
        hs = HostStreamEncoder(c, f, chunk=ch)
        ts = []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = hs.encode(host, f)
            ts.append(round((time.perf_counter() - t0) * 1e3, 3))
        out[f"chunk_{ch}_ms"] = ts
        print(json.dumps(out), flush=True)
        del hs
    out["packed_bytes"] = sum(r["bytes"])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
