"""Time so_pack_frames (and the D2H of its stream) on a 4K 30-frame GOP's symbols.
    python tools/pack_probe.py [--frames 30] [--reps 5]
Run it under `rocprofv3 --kernel-trace --stats` for the per-kernel split."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=30)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from streamoptima_amd.Encoder import Y_Video_codec
    from streamoptima_amd.engine import alloc_planes
    from streamoptima_amd.synth import synth_sequence_torch
    dev = torch.device("cuda:0")
    h, w, f = 2160, 3840, a.frames
    c = Y_Video_codec(h, w, f, 16, 16, 4, f, 0, 0.015, False, device=dev)
    fr = alloc_planes(f, h, w, dev)
    fr.copy_(synth_sequence_torch(f, h, w, seed=0, device=dev))
    syms = c.encode_device(fr, f)["symbols"]
    eng = c.engine()
    offs, out = eng.pack_symbols(syms)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(a.reps):
        e0.record()
        eng.pack_symbols(syms, offs, out)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    tot = offs[:, eng.nb].cpu().tolist()
    host = torch.empty(out.shape, dtype=torch.uint8).pin_memory()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i, n in enumerate(tot):
        host[i, :n].copy_(out[i, :n], non_blocking=True)
    torch.cuda.synchronize()
    d2h = time.perf_counter() - t0
    qtc_h = torch.empty((f,) + tuple(syms[0].qtc.shape), dtype=torch.int16).pin_memory()
    t0 = time.perf_counter()
    for i, s in enumerate(syms):
        qtc_h[i].copy_(s.qtc, non_blocking=True)
    torch.cuda.synchronize()
    d2h_dense = time.perf_counter() - t0
    print(json.dumps({"pack_ms": [round(t, 3) for t in ts], "packed_bytes": sum(tot),
                      "bytes_per_frame": round(sum(tot) / f), "d2h_packed_ms": round(d2h * 1e3, 3),
                      "d2h_packed_gbs": round(sum(tot) / d2h / 1e9, 2), "d2h_qtc_ms": round(d2h_dense * 1e3, 3),
                      "d2h_qtc_gbs": round(qtc_h.numel() * 2 / d2h_dense / 1e9, 2)}))


if __name__ == "__main__":
    main()
