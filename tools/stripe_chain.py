"""Per-frame time of the persistent P-frame run (so_encode_p_run) against frame height.

At N ranks a 4K stripe is 2160/N rows; with fewer tiles than resident workgroups the
frame-to-frame dependency chain, not throughput, sets the per-frame time.  This measures
that regime on ONE GPU: a 3840-wide frame of H rows, NF P-frames in persistent launches,
HIP events on the launch stream.

    python tools/stripe_chain.py [--heights 272,544,1088,2160] [--frames 60] [--width 3840]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--heights", default="272,544,1088,2160")
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--frames", type=int, default=60)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from streamoptima_amd.engine import Engine, alloc_planes
    from streamoptima_amd.synth import synth_sequence_torch
    dev = torch.device("cuda:0")
    out = {}
    for h in [int(x) for x in a.heights.split(",")]:
        eng = Engine(h, a.width, 16, 16, False, 0.015, dev)
        nf = a.frames + 1
        fr = alloc_planes(nf, h, a.width, dev)
        fr.copy_(synth_sequence_torch(nf, h, a.width, seed=0, device=dev))
        i0 = eng.encode_i(fr[0], 4)
        outs = [eng.new_symbols(1) for _ in range(nf - 1)]
        curs = [fr[i] for i in range(1, nf)]
        for _ in range(2):
            eng.encode_p_run(curs, i0.recon, 4, outs)
        st = torch.cuda.current_stream(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(st)
        for _ in range(a.reps):
            eng.encode_p_run(curs, i0.recon, 4, outs)
        e1.record(st)
        torch.cuda.synchronize()
        eng.check_run()
        us = e0.elapsed_time(e1) * 1e3 / a.reps / (nf - 1)
        tiles = (a.width // 128) * -(-h // 32)
        out[h] = {"per_frame_us": round(us, 2), "tiles_per_frame": tiles, "frames": nf - 1}
        print(f"H={h:5d} tiles/frame={tiles:5d}  {us:8.2f} us per P-frame", flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
