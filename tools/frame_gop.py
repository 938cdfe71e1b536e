"""Encode one 4K P-frame N times against the reconstruction of the previous P-frame (the
GOP's real workload: me_sea2_kernel + inter_tq_kernel), for rocprofv3 --pmc passes
(tools/gpu_pmc_gop.sh)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from streamoptima_amd.engine import Engine, alloc_planes  # noqa: E402
from streamoptima_amd.synth import synth_sequence_torch  # noqa: E402

h, w, n = 2160, 3840, int(os.environ.get("ME_N", 5))
dev = torch.device("cuda:0")
fr = alloc_planes(3, h, w, dev)
fr.copy_(synth_sequence_torch(3, h, w, 0, dev))
eng = Engine(h, w, 16, 16, False, 0.015, dev)
p1 = eng.encode_p(fr[1], [eng.encode_i(fr[0], 4).recon], 4)
sp = eng.new_symbols(1)
for _ in range(n):
    eng.encode_p(fr[2], [p1.recon], 4, out=sp)
torch.cuda.synchronize()
print("ok")
