"""A/B of ME implementations in one process (interleaved rounds), 4K P-frame.

Variants: me_sea2_kernel (default for bs 16 without VBS; with VBS the dense wave kernel) and
me_wave_kernel (SO_ME_IMPL=dense).  Checks every variant's output equals
the first one's, then prints us/launch per variant."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from streamoptima_amd import _lib
from streamoptima_amd.engine import alloc_planes
from streamoptima_amd.synth import synth_sequence_torch
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ab_guard import require_ab_build  # noqa: E402
require_ab_build()

VARIANTS = {"sea": {}, "dense": {"SO_ME_IMPL": "dense"}}


def main():
    h, w = int(os.environ.get("AB_H", 2160)), int(os.environ.get("AB_W", 3840))
    names = os.environ.get("AB_VARIANTS", ",".join(VARIANTS)).split(",")
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
        for rnd in range(3):
            for name in names:
                for k in ("SO_ME_READ", "SO_ME_IMPL"):
                    os.environ.pop(k, None)
                os.environ.update(VARIANTS[name])
                best = torch.empty((nb, 4), dtype=torch.int32, device=dev)
                sub = torch.empty((nb, 4, 4), dtype=torch.int32, device=dev) if vbs else None
                f = lambda: _lib.check(lib.so_me_full_search(fr[1].data_ptr(), refs, 1, h, w, 16, 16, best.data_ptr(),
                                                             _lib.ptr(sub), st), "me")
                for _ in range(3):
                    f()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(20):
                    f()
                e1.record()
                torch.cuda.synchronize()
                res.setdefault((vbs, name), []).append(e0.elapsed_time(e1) / 20 * 1e3)
                outs[name] = (best.cpu(), None if sub is None else sub.cpu())
        first = outs[names[0]]
        for name in names[1:]:
            same = torch.equal(outs[name][0], first[0]) and (not vbs or torch.equal(outs[name][1], first[1]))
            print(f"vbs={vbs} {name} identical_to_{names[0]}={same}")
    for k, v in res.items():
        print(f"vbs={k[0]} {k[1]:9s} us/launch: {['%.1f' % x for x in v]}  min {min(v):.1f}")


main()
