"""A/B of ME implementations in one process (interleaved rounds), 4K P-frame:
me_tile_kernel (default) vs me_fast_kernel (SO_ME_IMPL=fast, round-1 kernel)."""
import os, sys, time
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from streamoptima_amd import _lib
from streamoptima_amd.engine import alloc_planes
from streamoptima_amd.synth import synth_sequence_torch

def main():
    h, w = int(os.environ.get("AB_H", 2160)), int(os.environ.get("AB_W", 3840))
    dev = torch.device("cuda:0")
    lib = _lib.load()
    fr = alloc_planes(2, h, w, dev)
    fr.copy_(synth_sequence_torch(2, h, w, 1, dev))
    nb = (h // 16) * (w // 16)
    st = _lib.stream_handle()
    refs = _lib.ref_array([fr[0]])
    res = {}
    for vbs in (False, True):
        outs = {}
        for impl in ("tile", "fast", "tile", "fast", "tile", "fast"):
            os.environ["SO_ME_IMPL"] = impl
            best = torch.empty((nb, 4), dtype=torch.int32, device=dev)
            sub = torch.empty((nb, 4, 4), dtype=torch.int32, device=dev) if vbs else None
            f = lambda: _lib.check(lib.so_me_full_search(fr[1].data_ptr(), refs, 1, h, w, 16, 16, best.data_ptr(), _lib.ptr(sub), st), "me")
            for _ in range(3): f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize(); e0.record()
            for _ in range(20): f()
            e1.record(); torch.cuda.synchronize()
            res.setdefault((vbs, impl), []).append(e0.elapsed_time(e1) / 20 * 1e3)
            outs[impl] = (best.cpu().numpy(), None if sub is None else sub.cpu().numpy())
        same = (outs["tile"][0] == outs["fast"][0]).all() and (not vbs or (outs["tile"][1] == outs["fast"][1]).all())
        print(f"vbs={vbs} identical_outputs={same}")
    for k, v in res.items():
        print(f"vbs={k[0]} impl={k[1]:5s} us/launch: {['%.1f' % x for x in v]}  min {min(v):.1f}")

main()
