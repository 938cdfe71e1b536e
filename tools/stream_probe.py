"""Timeline of hoststream.encode_stream (4K x 30, 4 GOPs, two buffer sets): GPU event times of
each GOP's upload end, encode start / end and download end, relative to the first event.
    python tools/stream_probe.py [--nbuf 2] [--gops 4]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nbuf", type=int, default=2)
    ap.add_argument("--gops", type=int, default=4)
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
    hs = HostStreamEncoder(c, f, chunk=2, nbuf=a.nbuf)
    hs.encode_stream([host] * 2, f, lambda k, r: None)
    for rep in range(2):
        tr = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        hs.encode_stream([host] * a.gops, f, lambda k, r: None, trace=tr)
        wall = time.perf_counter() - t0
        torch.cuda.synchronize()
        e0 = tr[0][1]
        rows = [(lab, round(e0.elapsed_time(ev), 3), round((ht - t0) * 1e3, 3)) for lab, ev, ht in tr]
        rows.sort(key=lambda r: r[1])
        print(json.dumps({"rep": rep, "wall_ms_per_gop": round(wall / a.gops * 1e3, 3),
                          "events_gpu_ms_host_ms": rows}), flush=True)


if __name__ == "__main__":
    main()
