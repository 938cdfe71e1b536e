"""Per-workgroup phase stamps of me_sea2_kernel on the GOP's real workload (4K P-frame vs the
previous P-frame's reconstruction).  Needs the instrumented build:
    python -m streamoptima_amd.build --out tools/_ab/lib_stamps.so -D SO_STAMPS
    SO_LIB_PATH=tools/_ab/lib_stamps.so python tools/sea_stamps.py
Prints phase cycle statistics, the launch timeline (concurrent workgroups over time), per-XCD
spans and the survivor / fallback counts."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from streamoptima_amd import _lib  # noqa: E402
from streamoptima_amd.engine import Engine, alloc_planes  # noqa: E402
from streamoptima_amd.synth import synth_sequence_torch  # noqa: E402


def main():
    h, w = int(os.environ.get("STAMP_H", 2160)), int(os.environ.get("STAMP_W", 3840))
    dev = torch.device("cuda:0")
    lib = _lib.load()
    fr = alloc_planes(3, h, w, dev)
    fr.copy_(synth_sequence_torch(3, h, w, 0, dev))
    eng = Engine(h, w, 16, 16, False, 0.015, dev)
    p1 = eng.encode_p(fr[1], [eng.encode_i(fr[0], 4).recon], 4)
    torch.cuda.synchronize()
    ntiles = ((w // 16 + 7) // 8) * ((h // 16 + 1) // 2)
    stamps = torch.zeros((ntiles, 12), dtype=torch.int64, device=dev)
    lib.so_debug_set_sea_stamps.argtypes = [ctypes.c_void_p]
    assert lib.so_debug_set_sea_stamps(stamps.data_ptr()) == 0
    nb = (h // 16) * (w // 16)
    best = torch.empty((nb, 4), dtype=torch.int32, device=dev)
    refs = _lib.ref_array([p1.recon])
    fused = os.environ.get("STAMP_FUSED", "0") == "1"    # p_tile_kernel (ME + transforms) instead
    sp = eng.new_symbols(1)
    for _ in range(int(os.environ.get("REPS", 5))):
        if fused:
            eng.encode_p(fr[2], [p1.recon], 4, out=sp)
        else:
            _lib.check(lib.so_me_full_search(fr[2].data_ptr(), refs, 1, h, w, 16, 16, best.data_ptr(), None,
                                             _lib.stream_handle()), "me")
    torch.cuda.synchronize()
    s = stamps.cpu().numpy().astype(np.int64)
    rt0, rt1 = s[:, 0], s[:, 7]
    cyc = s[:, 6] - s[:, 1]
    span_rt = (rt1.max() - rt0.min()) * 10e-3          # us (100 MHz)
    ghz = (cyc / np.maximum((rt1 - rt0) * 10e-9, 1e-12)).mean() / 1e9
    print(f"tiles {ntiles}  kernel span (first start -> last end) {span_rt:.1f} us  shader clock ~{ghz:.2f} GHz")
    names = ["cur+a4", "window", "b4 sums", "search", "epilogue" + (" (records + transforms)" if fused else "")]
    for i, n in enumerate(names):
        d = s[:, i + 2] - s[:, i + 1]
        print(f"  {n:9s} cycles mean {d.mean():8.0f}  p50 {np.median(d):8.0f}  p90 {np.percentile(d, 90):8.0f}  "
              f"max {d.max():8.0f}  ({d.mean() / cyc.mean() * 100:4.1f}%)")
    print(f"  total     cycles mean {cyc.mean():8.0f}  p50 {np.median(cyc):8.0f}  max {cyc.max():8.0f}  "
          f"= {cyc.mean() / ghz / 1e3:.2f} us per workgroup")
    fb = s[:, 9] >> 32
    sur = s[:, 9] & 0xFFFFFFFF
    print(f"  fallback blocks {fb.sum()} of {nb} ({fb.sum() / nb * 100:.2f}%)  survivors mean/block "
          f"{sur.sum() / nb:.1f}; tiles with a fallback {np.mean(fb > 0) * 100:.1f}%")
    # timeline: concurrent workgroups
    t0 = rt0.min()
    ev = np.concatenate([np.stack([rt0 - t0, np.ones_like(rt0)], 1), np.stack([rt1 - t0, -np.ones_like(rt1)], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    conc = np.cumsum(ev[:, 1])
    tt = ev[:, 0]
    dur = np.diff(tt, append=tt[-1])
    tot = dur.sum()
    mx = conc.max()
    print(f"  max concurrent workgroups {mx}; time-weighted mean {np.sum(conc * dur) / max(tot, 1):.0f}")
    for frac in (1.0, 0.75, 0.5, 0.25):
        print(f"    time with >= {frac:4.2f} x max concurrent: {np.sum(dur[conc >= frac * mx]) / max(tot, 1) * 100:5.1f}%")
    order = np.argsort(rt0)
    print("  start times (us) of workgroup deciles:",
          " ".join(f"{(rt0[order[int(q * (ntiles - 1))]] - t0) * 1e-2:.1f}" for q in np.linspace(0, 1, 11)))
    print("  end times (us) deciles:", " ".join(f"{x * 1e-2:.1f}" for x in np.percentile(rt1 - t0, np.linspace(0, 100, 11))))
    xcc = s[:, 8] >> 32
    for x in np.unique(xcc):
        m = xcc == x
        print(f"  xcc {x}: tiles {m.sum():4d}  start {(rt0[m].min() - t0) * 1e-2:5.1f}  end {(rt1[m].max() - t0) * 1e-2:5.1f} us"
              f"  mean cycles {cyc[m].mean():.0f}")


if __name__ == "__main__":
    main()
