"""Run one ME implementation (SO_ME_IMPL) on a 4K P-frame N times (for rocprofv3 --pmc)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from streamoptima_amd import _lib
from streamoptima_amd.engine import alloc_planes
from streamoptima_amd.synth import synth_sequence_torch
h, w, n = 2160, 3840, int(os.environ.get("ME_N", 10))
vbs = os.environ.get("ME_VBS", "0") == "1"
dev = torch.device("cuda:0")
lib = _lib.load()
fr = alloc_planes(2, h, w, dev); fr.copy_(synth_sequence_torch(2, h, w, 1, dev))
nb = (h // 16) * (w // 16)
best = torch.empty((nb, 4), dtype=torch.int32, device=dev)
sub = torch.empty((nb, 4, 4), dtype=torch.int32, device=dev) if vbs else None
refs = _lib.ref_array([fr[0]])
for _ in range(n):
    _lib.check(lib.so_me_full_search(fr[1].data_ptr(), refs, 1, h, w, 16, 16, best.data_ptr(), _lib.ptr(sub), _lib.stream_handle()), "me")
torch.cuda.synchronize()
print("ok", os.environ.get("SO_ME_IMPL", "qsad"))
