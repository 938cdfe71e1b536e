"""Copy-engine rates behind BASELINE.md §4's region (diagnostic): the 4K GOP's 30 Y planes
(249 MB) uploaded from a registered host buffer (hostmem.pinned_empty) on a dedicated stream
as one copy, one copy per 2 / 1 frames (with an event after each, as hoststream does), alone
and with the packed streams' download (6.8 MB per frame, one copy per 2 frames) running the
other way on a second dedicated stream.  GPU-event times, median of 6 after 2 warm-up runs.
    python tools/s4_links.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from streamoptima_amd.hostmem import pinned_empty
    from streamoptima_amd.hwqueue import dedicated_stream
    dev = torch.device("cuda:0")
    f, fb, pb = 30, 2160 * 3840, 6_823_865
    hu = pinned_empty((f, fb))
    hu.fill_(3)
    du = torch.empty((f, fb), dtype=torch.uint8, device=dev)
    dd = torch.zeros((f, pb), dtype=torch.uint8, device=dev)
    hd = pinned_empty((f, pb))
    sa, sb = dedicated_stream(dev, "probe.h2d"), dedicated_stream(dev, "probe.d2h")

    def up(g):
        with torch.cuda.stream(sa):
            for i in range(0, f, g):
                du[i:i + g].copy_(hu[i:i + g], non_blocking=True)
                torch.cuda.Event().record(sa)

    def down(g=2):
        with torch.cuda.stream(sb):
            for i in range(0, f, g):
                hd[i:i + g].copy_(dd[i:i + g], non_blocking=True)

    def timed(fn, n=8):
        ts = []
        for _ in range(n):
            torch.cuda.synchronize()
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            cur = torch.cuda.current_stream(dev)
            e0.record(cur)
            sa.wait_stream(cur)
            sb.wait_stream(cur)
            fn()
            e1.record(sa)
            e2.record(sb)
            torch.cuda.synchronize()
            ts.append((e0.elapsed_time(e1), e0.elapsed_time(e2)))
        ts = sorted(ts[2:])
        return [round(v, 3) for v in ts[len(ts) // 2]]

    out = {}
    for g in (30, 10, 2, 1):
        a = timed(lambda g=g: up(g))[0]
        out[f"up_g{g}"] = {"ms": a, "GBs": round(f * fb / a / 1e6, 2)}
        b = timed(lambda g=g: (up(g), down()))
        out[f"up_g{g}+down"] = {"up_ms": b[0], "down_ms": b[1], "up_GBs": round(f * fb / b[0] / 1e6, 2)}
    d = timed(down)[1]
    out["down_g2"] = {"ms": d, "GBs": round(f * pb / d / 1e6, 2)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
