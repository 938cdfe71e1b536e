"""p_run_kernel tile width A/B (SO_RUN_TPX): per-frame time of a persistent P-run at 4K and
1088p with 128- and 64-px tiles.   python tools/tpx_ab.py"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from streamoptima_amd.engine import Engine, alloc_planes
    from streamoptima_amd.synth import synth_sequence_torch
    dev = torch.device("cuda:0")
    out = {}
    for h in (2160, 1088, 544, 272):
        w, f = 3840 if h != 1088 else 1920, 30
        eng = Engine(h, w, 16, 16, False, 0.015, dev)
        fr = alloc_planes(f, h, w, dev)
        fr.copy_(synth_sequence_torch(f, h, w, seed=0, device=dev))
        i0 = eng.encode_i(fr[0], 4)
        outs = [eng.new_symbols(1) for _ in range(f - 1)]
        for tpx in ("128", "64"):
            os.environ["SO_RUN_TPX"] = tpx
            best = None
            for _ in range(6):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                eng.encode_p_run([fr[i] for i in range(1, f)], i0.recon, 4, outs)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                best = dt if best is None else min(best, dt)
            eng.check_run()
            out[f"{w}x{h}_tpx{tpx}_us_per_frame"] = round(best / (f - 1) * 1e6, 2)
            print(json.dumps(out), flush=True)
    os.environ.pop("SO_RUN_TPX", None)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
