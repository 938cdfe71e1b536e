"""VBS split statistics of the bench content (GPU): how many blocks could skip the sub-block
transforms because the split is decided before them.

The RD decision (Encoder.py:564-578, calculate_RD_cost :1133-1158) splits a block iff
c_v <= c_b, c = lam * bits + mae.  The sub-block token count is at least 4 (four end markers),
so c_v >= lam * (64 + 32) + mae_v, and a block with c_b below that bound can never split -- its
four 8x8 transforms only feed a decision already made.  With SAD_b >= sum SAD_j (mae_b >=
mae_v) the bound needs c_b < lam * 96 + mae_v, i.e. for an unsplit block
lam * (16 + 8 tok_b) + (SAD_b - sum SAD_j) / 256 < lam * 96: this counts the unsplit blocks with
lam * (16 + 8 tok_b) < lam * 96 (tok_b < 10), an upper bound on the skippable share.

    python tools/vbs_split_stats.py   (on the GPU box)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from streamoptima_amd.engine import Engine, alloc_planes
    from streamoptima_amd.synth import synth_sequence_torch
    h, w, f = 2160, 3840, 4
    dev = torch.device("cuda:0")
    eng = Engine(h, w, 16, 16, True, 0.015, dev)
    fr = alloc_planes(f, h, w, dev)
    fr.copy_(synth_sequence_torch(f, h, w, seed=0, device=dev, content=os.environ.get("SO_AB_CONTENT", "bench")))
    ref = eng.encode_i(fr[0], 4).recon
    for i in range(1, f):
        s = eng.encode_p(fr[i], [ref], 4)
        torch.cuda.synchronize()
        split = s.split.cpu().numpy().astype(bool)
        tok = s.tokens.cpu().numpy()
        uns = ~split
        print(f"frame {i}: split {split.mean():.3f}; unsplit blocks with tok_b < 10: {(uns & (tok < 10)).mean():.3f} "
              f"of all blocks; unsplit token median {int(torch.tensor(tok[uns]).median()) if uns.any() else -1}")
        ref = s.recon


if __name__ == "__main__":
    main()
