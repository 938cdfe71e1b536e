"""Run the 4K P-frame path (so_encode_p_frame: ME + TQ) and one I-frame N times, for
rocprofv3 --pmc passes (tools/gpu_pmc.sh).  ME_VBS=1 for the VBS variant."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from streamoptima_amd.engine import Engine, alloc_planes  # noqa: E402
from streamoptima_amd.synth import synth_sequence_torch  # noqa: E402

h, w, n = 2160, 3840, int(os.environ.get("ME_N", 5))
vbs = os.environ.get("ME_VBS", "0") == "1"
dev = torch.device("cuda:0")
fr = alloc_planes(2, h, w, dev)
fr.copy_(synth_sequence_torch(2, h, w, 1, dev))
eng = Engine(h, w, 16, 16, vbs, 0.015, dev)
sp, si = eng.new_symbols(1), eng.new_symbols(0)
for _ in range(n):
    eng.encode_p(fr[1], [fr[0]], 4, out=sp)
    eng.encode_i(fr[1], 4, out=si)
torch.cuda.synchronize()
print("ok vbs", vbs)
