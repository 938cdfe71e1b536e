"""Compare the stripe run (pipeline.StripeRunRank, in-process ranks) with the one-GPU GOP
array by array (debugging aid)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from streamoptima_amd.engine import Engine, alloc_planes
    from streamoptima_amd.Encoder import Y_Video_codec
    from streamoptima_amd.pipeline import StripeRunRank
    from streamoptima_amd.synth import synth_sequence_torch
    dev = torch.device("cuda:0")
    h, w, nf, world = (int(os.environ.get("H", 1088)), int(os.environ.get("W", 1920)), int(os.environ.get("NF", 3)),
                        int(os.environ.get("WORLD", 2)))
    fr = alloc_planes(nf, h, w, dev)
    fr.copy_(synth_sequence_torch(nf, h, w, seed=0, device=dev))
    codec = Y_Video_codec(h, w, nf, 16, 16, 4, nf, 0, 0.015, False, device=dev)
    ref = codec.encode_device(fr, nf)["symbols"]
    torch.cuda.synchronize()
    engines = [Engine(h, w, 16, 16, False, 0.015, dev) for _ in range(world)]
    streams = [torch.cuda.Stream(dev) for _ in range(world)]
    ranks = [StripeRunRank(engines[r], world, r, nf, stream=streams[r], max_wg=768 // (2 * world)) for r in range(world)]
    torch.cuda.synchronize()
    for r in range(world):
        ranks[r].connect(ranks[r - 1].info() if r > 0 else None, ranks[r + 1].info() if r < world - 1 else None)
    for rep in range(int(os.environ.get("REPS", 1))):
        syms = []
        for r in range(world):
            with torch.cuda.stream(streams[r]):
                syms.append(ranks[r].encode(fr, nf, 4))
        torch.cuda.synchronize()
        for r in ranks:
            print("rep", rep, "timed out:", r.timed_out(), "stripe", r.by0, r.by1, flush=True)
    nbx = w // 16
    for i in range(nf):
        for k in ("split", "mv", "qtc", "tokens", "mae_num"):
            got = np.concatenate([getattr(s[i], k).cpu().numpy() for s in syms])
            exp = getattr(ref[i], k).cpu().numpy()
            bad = np.argwhere(got != exp) if got.shape == exp.shape else None
            if bad is None:
                print(i, k, "shape", got.shape, exp.shape)
            elif len(bad):
                blocks = sorted(set((b[0] // nbx) for b in bad))
                print(i, k, len(bad), "mismatches; block rows", blocks[:10], "first", bad[:3].tolist())
        rec = np.concatenate([r.stripe_recon(i).cpu().numpy() for r in ranks])
        exp = ref[i].recon.cpu().numpy()
        bad = np.argwhere(rec != exp)
        if len(bad):
            print(i, "recon", len(bad), "mismatches; rows", sorted(set(bad[:, 0].tolist()))[:20])
    print("done")


if __name__ == "__main__":
    main()
