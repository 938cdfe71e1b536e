"""Offline analysis (test infrastructure: the C oracle supplies the reconstructions): survivors
of an exact 8x8-cell bound (sum over 4 cells of |S8_cur - S8_ref|, 16-bit sums, no
quantisation slack) when U is the best SAD among predicted candidates -- the co-located
block's MV in the previous P-frame and (0, 0) -- instead of the SAD of the smallest 4x4 bound.
    python tests/analysis/sea_mv_pred.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle import oracle as O  # noqa: E402
from streamoptima_amd.synth import synth_sequence  # noqa: E402


def boxsum(a, k):
    c = np.zeros((a.shape[0] + 1, a.shape[1] + 1), np.int64)
    c[1:, 1:] = a.cumsum(0).cumsum(1)
    return c[k:, k:] - c[:-k, k:] - c[k:, :-k] + c[:-k, :-k]


def main(h=272, w=480, seed=0):
    seq = synth_sequence(4, h, w, seed=seed)
    i0 = O.intra_frame(seq[0], 16, 16, 4)
    p1 = O.inter_frame(seq[1], [i0["recon"]], 16, 16, 4)
    prev_mv = p1["mv"][:, 0, :2].reshape(h // 16, w // 16, 2)       # frame 1's MVs
    ref = p1["recon"].astype(np.int64)
    cur = seq[2].astype(np.int64)
    B8 = boxsum(ref, 8)
    surv, hit = [], 0
    for by in range(h // 16):
        for bx in range(w // 16):
            x, y = bx * 16, by * 16
            blk = cur[y:y + 16, x:x + 16]
            A8 = blk.reshape(2, 8, 2, 8).sum(axis=(1, 3))
            cands, sads, lbs = [], [], []
            for dx in range(-16, 17):
                for dy in range(-16, 17):
                    if not (0 <= x + dx < w - 16 and 0 <= y + dy < h - 16):
                        continue
                    cands.append((dx, dy))
                    lbs.append(np.abs(A8 - B8[y + dy:y + dy + 16:8, x + dx:x + dx + 16:8]).sum())
                    sads.append(np.abs(blk - ref[y + dy:y + dy + 16, x + dx:x + dx + 16]).sum())
            if not cands:
                continue
            sads, lbs = np.array(sads), np.array(lbs)
            idx = {c: i for i, c in enumerate(cands)}
            preds = [tuple(prev_mv[by, bx]), (0, 0)]
            u = min(sads[idx[p]] for p in preds if p in idx) if any(p in idx for p in preds) else sads.max()
            hit += u == sads.min()
            surv.append(int((lbs <= u).sum()))
    a = np.array(surv)
    print(f"seed {seed}: blocks {a.size}, U = true min for {hit / a.size:.3f}; survivors mean {a.mean():.1f} "
          f"median {np.median(a):.0f} p90 {np.percentile(a, 90):.0f} p99 {np.percentile(a, 99):.0f} max {a.max()} "
          f">16 {(a > 16).mean():.3f} >64 {(a > 64).mean():.3f}")


if __name__ == "__main__":
    main(seed=0)
    main(seed=1)
