"""Offline analysis (test infrastructure: the C oracle supplies the reconstructions): the sizes of
sea_vbs_block's two survivor lists (so_me.hip) on the bench texture, with the kernel's quantised
bounds -- list A (block bound <= U) and list B (some sub-block bound <= U_j, not in A) -- and how
many of the four sub-blocks pass per list-B candidate (list B evaluates all four today).
    python tests/analysis/sea_vbs_lists.py [h w]"""
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
    seq = synth_sequence(3, h, w, seed=seed)
    i0 = O.intra_frame(seq[0], 16, 16, 4)
    p1 = O.inter_frame(seq[1], [i0["recon"]], 16, 16, 4)
    ref = p1["recon"].astype(np.int64)
    cur = seq[2].astype(np.int64)
    q4 = boxsum(ref, 4) >> 4            # q of every 4x4 cell position of the reference
    nA, nB, quads = [], [], []
    for by in range(1, h // 16 - 2):
        for bx in range(1, w // 16 - 2):
            x, y = bx * 16, by * 16
            if x + 48 > w or y + 48 > h or x < 16 or y < 16:
                continue
            blk = cur[y:y + 16, x:x + 16]
            a4 = blk.reshape(4, 4, 4, 4).sum(axis=(1, 3)) >> 4
            sub, lbj = [], []
            for dy in range(-16, 17):
                for dx in range(-16, 17):
                    d = np.abs(blk - ref[y + dy:y + dy + 16, x + dx:x + dx + 16])
                    sub.append([d[:8, :8].sum(), d[:8, 8:].sum(), d[8:, :8].sum(), d[8:, 8:].sum()])
                    c4 = np.abs(a4 - q4[y + dy:y + dy + 16:4, x + dx:x + dx + 16:4])
                    lbj.append([c4[:2, :2].sum(), c4[:2, 2:].sum(), c4[2:, :2].sum(), c4[2:, 2:].sum()])
            sub, lbj = np.array(sub), np.array(lbj)
            full, lb = sub.sum(1), lbj.sum(1)
            U = full[np.argmin(lb)]
            inA = lb <= (U + 240) >> 4
            uj = sub[inA].min(0)
            passj = lbj <= ((uj + 60) >> 4)[None, :]
            inB = passj.any(1) & ~inA
            nA.append(int(inA.sum()))
            nB.append(int(inB.sum()))
            if inB.any():
                quads.extend(passj[inB].sum(1).tolist())
    nA, nB, quads = np.array(nA), np.array(nB), np.array(quads)
    print(f"blocks {nA.size}: list A mean {nA.mean():.1f} median {np.median(nA):.0f} p90 {np.percentile(nA, 90):.0f}; "
          f"list B mean {nB.mean():.1f} median {np.median(nB):.0f} p90 {np.percentile(nB, 90):.0f} "
          f"(> 384: {(nB > 384).mean():.3f}, A > 384: {(nA > 384).mean():.3f})")
    print("sub-blocks passing per list-B candidate: " +
          ", ".join(f"{k}: {(quads == k).mean():.3f}" for k in range(1, 5)) + f"; mean {quads.mean():.2f}")


if __name__ == "__main__":
    a = [int(v) for v in sys.argv[1:3]]
    main(*a) if a else main()
