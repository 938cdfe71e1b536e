"""ME launch time vs. frame height (number of workgroup tiles) on the GOP's real workload:
the 4K P-frame searched against the previous reconstruction, cropped to the first H rows.
Separates per-tile cost from launch / tail effects (tools/me_ab2.py has the variants)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from streamoptima_amd import _lib  # noqa: E402
from streamoptima_amd.engine import Engine, alloc_planes  # noqa: E402
from streamoptima_amd.synth import synth_sequence_torch  # noqa: E402


def main():
    h, w = 2160, 3840
    heights = [int(x) for x in os.environ.get("ME_HEIGHTS", "512,800,1024,1600,2048,2160").split(",")]
    dev = torch.device("cuda:0")
    lib = _lib.load()
    fr = alloc_planes(3, h, w, dev)
    fr.copy_(synth_sequence_torch(3, h, w, 0, dev))
    eng = Engine(h, w, 16, 16, False, 0.015, dev)
    i0 = eng.encode_i(fr[0], 4)
    p1 = eng.encode_p(fr[1], [i0.recon], 4)
    cur, ref = fr[2], p1.recon
    st = _lib.stream_handle()
    refs = _lib.ref_array([ref])
    for hh in heights:
        nb = (hh // 16) * (w // 16)
        best = torch.empty((nb, 4), dtype=torch.int32, device=dev)
        f = lambda: _lib.check(lib.so_me_full_search(cur.data_ptr(), refs, 1, hh, w, 16, 16, best.data_ptr(),  # noqa: E731
                                                     None, st), "me")
        ts = []
        for _ in range(3):
            for _ in range(2):
                f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(10):
                f()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 10 * 1e3)
        tiles = -(-(hh // 16) // 2) * -(-(w // 16) // 8)
        print(f"H={hh:5d} tiles={tiles:5d} us/launch min {min(ts):6.1f}  us/tile*768 {min(ts) / tiles * 768:6.2f}", flush=True)


if __name__ == "__main__":
    main()
