"""Timeline of BASELINE.md §4's region as bench.py times it (hoststream.HostStreamEncoder.encode,
4K x 30, one buffer set, chunk 2): per P-run chunk, when the compute stream starts it (its
frames uploaded), when its pack ends, when its download starts, and the host time at which each
of those was enqueued -- so a compute stream waiting on the host, or a download waiting on the
host's byte-count read, shows as a gap.
    python tools/s4_timeline.py [--chunk 2] [--reps 4] [--upload chunk|frame] [--quiet]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunk", type=int, default=2)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--upload", default="chunk")
    ap.add_argument("--quiet", action="store_true")
    a = ap.parse_args()
    from streamoptima_amd.Encoder import Y_Video_codec
    from streamoptima_amd.engine import alloc_planes
    from streamoptima_amd.hostmem import pinned_empty
    from streamoptima_amd.hoststream import HostStreamEncoder
    from streamoptima_amd.synth import synth_sequence_torch
    dev = torch.device("cuda:0")
    h, w, f = 2160, 3840, 30
    c = Y_Video_codec(h, w, f, 16, 16, 4, f, 0, 0.015, False, device=dev)
    fr = alloc_planes(f, h, w, dev)
    fr.copy_(synth_sequence_torch(f, h, w, seed=0, device=dev))
    host = pinned_empty(tuple(fr.shape))
    host.copy_(fr.cpu())
    hs = HostStreamEncoder(c, f, chunk=a.chunk, upload=a.upload)
    for _ in range(2):
        hs.encode(host, f)
    walls = []
    for rep in range(a.reps):
        tr = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record(torch.cuda.current_stream(dev))
        hs.encode_stream([host], f, lambda k, r: None, trace=None if a.quiet else tr)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        walls.append(wall * 1e3)
        if a.quiet:
            continue
        rows = {}
        for lab, ev, ht in tr:
            rows[lab] = (round(e0.elapsed_time(ev), 3), round((ht - t0) * 1e3, 3))
        # per chunk: go / end on the compute stream, download start, each with its host enqueue time
        ch = []
        for k0 in range(1, f, a.chunk):
            g, e, d = rows.get(f"chunk_go {k0}"), rows.get(f"chunk_end {k0}"), rows.get(f"d2h_go {k0}")
            ch.append([k0, g, e, d])
        print(json.dumps({"rep": rep, "wall_ms": round(wall * 1e3, 3), "up_end": rows.get("up_end 0"),
                          "enc_start": rows.get("enc_start 0"), "enc_end": rows.get("enc_end 0"),
                          "d2h_end": rows.get("d2h_end 0"),
                          "chunks[k0, go(gpu,host), end(gpu,host), d2h_go(gpu,host)]": ch}), flush=True)
    walls.sort()
    print(json.dumps({"chunk": a.chunk, "upload": a.upload, "wall_ms_min": round(walls[0], 3),
                      "wall_ms_median": round(walls[len(walls) // 2], 3)}), flush=True)


if __name__ == "__main__":
    main()
