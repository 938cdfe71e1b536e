"""Share of blocks whose matrix-core forward transform fails its certificate (fwd_mfma) and
takes the FP64 forward: run with SO_LIB_PATH = a -DSO_FWD_MFMA=1 -DSO_FWD_COUNT build, whose
kernels put the flagged-block count where the SAD count goes (words 66..67)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from streamoptima_amd.engine import Engine, alloc_planes  # noqa: E402
from streamoptima_amd.synth import synth_sequence_torch  # noqa: E402

dev = torch.device("cuda:0")
out = {}
for (h, w), content in (((2160, 3840), "bench"), ((1088, 1920), "bench"), ((2160, 3840), "lowtex"),
                        ((2160, 3840), "noise")):
    f = 8
    eng = Engine(h, w, 16, 16, False, 0.015, dev)
    fr = alloc_planes(f, h, w, dev)
    fr.copy_(synth_sequence_torch(f, h, w, seed=0, device=dev, content=content))
    i0 = eng.encode_i(fr[0], 4)
    outs = [eng.new_symbols(1) for _ in range(f - 1)]
    eng.take_sad_ops()
    eng.encode_p_run([fr[i] for i in range(1, f)], i0.recon, 4, outs)
    torch.cuda.synchronize()
    eng.check_run()
    n = eng.take_sad_ops()
    out[f"{w}x{h}_{content}"] = {"flagged": n, "blocks": eng.nb * (f - 1), "share": round(n / (eng.nb * (f - 1)), 4)}
print(json.dumps(out))
