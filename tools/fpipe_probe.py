"""Cost of the frame pipeline's mechanism on ONE GPU: a GOP through N in-process ranks, each
with 1/N of the machine's resident workgroups, against the one-rank persistent run with
the same total (uncached landing-plane reads, per-tile push + flag, cross-rank waits; no
xGMI).  Per-frame time of each, 4K.
    python tools/fpipe_probe.py [--frames 24] [--worlds 1,2,3]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=24)
    ap.add_argument("--worlds", default="2,3")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--height", type=int, default=2160)
    a = ap.parse_args()
    from streamoptima_amd.engine import Engine, alloc_planes
    from streamoptima_amd.pipeline import FramePipeRank
    from streamoptima_amd.synth import synth_sequence_torch
    dev = torch.device("cuda:0")
    h, w, f = a.height, 3840, a.frames
    fr = alloc_planes(f, h, w, dev)
    fr.copy_(synth_sequence_torch(f, h, w, seed=0, device=dev))
    out = {}
    # one rank: I-frame + one persistent run, whole machine
    eng = Engine(h, w, 16, 16, False, 0.015, dev)
    i0 = eng.encode_i(fr[0], 4)
    outs = [eng.new_symbols(1) for _ in range(f - 1)]

    def one():
        eng.encode_i(fr[0], 4, out=i0)
        eng.encode_p_run([fr[i] for i in range(1, f)], i0.recon, 4, outs)
    best = None
    for _ in range(a.reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        one()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    eng.check_run()
    out["one_rank_us_per_frame"] = round(best / f * 1e6, 2)
    streams = [torch.cuda.Stream(dev) for _ in range(3)]
    for world in [int(x) for x in a.worlds.split(",")]:
        cap = 768 // world
        engines = [Engine(h, w, 16, 16, False, 0.015, dev) for _ in range(world)]
        ranks = [FramePipeRank(engines[r], world, r, f, stream=streams[r], max_wg=cap) for r in range(world)]
        torch.cuda.synchronize()
        for r in range(world):
            ranks[r].connect(ranks[(r + 1) % world].info(), ranks[(r - 1) % world].info())
        best = None
        for _ in range(a.reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for r in range(world):
                with torch.cuda.stream(streams[r]):
                    ranks[r].encode(fr, f, 4)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        for r in ranks:
            r.check()
            r.close()
        out[f"fpipe_{world}_ranks_us_per_frame"] = round(best / f * 1e6, 2)
        print(json.dumps(out), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
