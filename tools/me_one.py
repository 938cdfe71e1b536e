"""Run one ME implementation (SO_ME_IMPL) N times on a 4K P-frame searched against the
reconstruction of the previous P-frame (the GOP's real workload), for rocprofv3 --pmc."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from streamoptima_amd import _lib
from streamoptima_amd.engine import Engine, alloc_planes
from streamoptima_amd.synth import synth_sequence_torch
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ab_guard import require_ab_build  # noqa: E402
require_ab_build()
h, w, n = 2160, 3840, int(os.environ.get("ME_N", 10))
vbs = os.environ.get("ME_VBS", "0") == "1"
dev = torch.device("cuda:0")
lib = _lib.load()
fr = alloc_planes(3, h, w, dev); fr.copy_(synth_sequence_torch(3, h, w, 0, dev))
impl = os.environ.pop("SO_ME_IMPL", None)        # the recon chain uses the default path
eng = Engine(h, w, 16, 16, False, 0.015, dev)
p1 = eng.encode_p(fr[1], [eng.encode_i(fr[0], 4).recon], 4)
torch.cuda.synchronize()
if impl:
    os.environ["SO_ME_IMPL"] = impl
nb = (h // 16) * (w // 16)
best = torch.empty((nb, 4), dtype=torch.int32, device=dev)
sub = torch.empty((nb, 4, 4), dtype=torch.int32, device=dev) if vbs else None
refs = _lib.ref_array([p1.recon])
for _ in range(n):
    _lib.check(lib.so_me_full_search(fr[2].data_ptr(), refs, 1, h, w, 16, 16, best.data_ptr(), _lib.ptr(sub), _lib.stream_handle()), "me")
torch.cuda.synchronize()
print("ok", impl or "default")
