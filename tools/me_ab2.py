"""ME A/B on the GOP's real workload: a 4K P-frame searched against the reconstruction of
the previous frame (I-frame recon, then a P recon), like bench.py's roofline launches.
Variants by environment (SO_ME_IMPL, SO_SEA_PROBE timing probes); prints us/launch and
checks the non-probe variants agree."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from streamoptima_amd import _lib  # noqa: E402
from streamoptima_amd.engine import Engine, alloc_planes  # noqa: E402
from streamoptima_amd.synth import synth_sequence_torch  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ab_guard import require_ab_build  # noqa: E402
require_ab_build()

VARIANTS = {"sea": {}, "dense": {"SO_ME_IMPL": "dense"}, "probe_stage": {"SO_SEA_PROBE": "1"},
            "probe_bounds": {"SO_SEA_PROBE": "2"}, "probe_nofallback": {"SO_SEA_PROBE": "3"},
            "probe_list": {"SO_SEA_PROBE": "4"}}


def main():
    h, w = 2160, 3840
    names = os.environ.get("AB_VARIANTS", ",".join(VARIANTS)).split(",")
    dev = torch.device("cuda:0")
    lib = _lib.load()
    fr = alloc_planes(3, h, w, dev)
    fr.copy_(synth_sequence_torch(3, h, w, 0, dev))
    eng = Engine(h, w, 16, 16, False, 0.015, dev)
    i0 = eng.encode_i(fr[0], 4)
    p1 = eng.encode_p(fr[1], [i0.recon], 4)
    pairs = [(fr[1], i0.recon), (fr[2], p1.recon)]
    nb = eng.nb
    st = _lib.stream_handle()
    res, outs = {}, {}
    for rnd in range(3):
        for name in names:
            for k in ("SO_ME_IMPL", "SO_SEA_PROBE"):
                os.environ.pop(k, None)
            os.environ.update(VARIANTS[name])
            for pi, (cur, ref) in enumerate(pairs):
                best = torch.empty((nb, 4), dtype=torch.int32, device=dev)
                refs = _lib.ref_array([ref])
                f = lambda: _lib.check(lib.so_me_full_search(cur.data_ptr(), refs, 1, h, w, 16, 16, best.data_ptr(),  # noqa: E731
                                                             None, st), "me")
                for _ in range(2):
                    f()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(10):
                    f()
                e1.record()
                torch.cuda.synchronize()
                res.setdefault((name, pi), []).append(e0.elapsed_time(e1) / 10 * 1e3)
                outs[(name, pi)] = best.cpu()
    for pi in range(len(pairs)):
        for name in names:
            if not name.startswith("probe") and name != names[0]:
                print(f"pair {pi} {name} identical_to_{names[0]}={bool((outs[(name, pi)] == outs[(names[0], pi)]).all())}")
        for name in names:
            v = res[(name, pi)]
            print(f"pair {pi} {name:14s} us/launch: {['%.1f' % x for x in v]}  min {min(v):.1f}")


if __name__ == "__main__":
    main()
