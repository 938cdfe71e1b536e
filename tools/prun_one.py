"""One workload's P-run replayed a few times (for rocprofv3 --pmc passes over a library
variant): 4K (or SO_AB_SIZE=HxW) 30-frame GOP content, the 29 P-frames as one persistent run
(Engine.encode_p_run), REPS times.  SO_LIB_PATH selects an A/B library, SO_AB_VBS=1 VBSEnable,
SO_AB_CONTENT the synth content."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from streamoptima_amd.engine import Engine, alloc_planes  # noqa: E402
from streamoptima_amd.synth import synth_sequence_torch  # noqa: E402

h, w = (int(v) for v in os.environ.get("SO_AB_SIZE", "2160x3840").split("x"))
f = 30
dev = torch.device("cuda:0")
eng = Engine(h, w, 16, 16, os.environ.get("SO_AB_VBS") == "1", 0.015, dev)
fr = alloc_planes(f, h, w, dev)
fr.copy_(synth_sequence_torch(f, h, w, seed=0, device=dev, content=os.environ.get("SO_AB_CONTENT", "bench")))
i0 = eng.encode_i(fr[0], 4)
outs = [eng.new_symbols(1) for _ in range(f - 1)]
for _ in range(int(os.environ.get("REPS", "4"))):
    eng.encode_p_run([fr[i] for i in range(1, f)], i0.recon, 4, outs)
torch.cuda.synchronize()
eng.check_run()
print("ok")
