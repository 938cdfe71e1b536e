"""Offline analysis (test infrastructure: uses the C oracle, so it lives under tests/).
Survivors of the exact SEA bound (16 LBq - 240 <= U, the kernels' quantised 4x4 sums) per
block of a 3840-wide strip of the bench content, for P-frame F (reference = the oracle's
reconstruction chain I, P1, ..., P(F-1)), under choices of U: the SAD of the smallest-bound
candidate (`cur`, sea2_tile's first count), the least SAD among the 4 smallest bounds
(`top4`), among each quadrant's smallest bound (`quad`), the 16 smallest, and the block
minimum (`ideal`, the floor any U can reach).  Usage: python tests/analysis/sea_refine.py F
"""
import numpy as np, sys
sys.path.insert(0, "/root/repo")
from streamoptima_amd.synth import synth_sequence
from oracle import oracle as O
h, w = 160, 3840
seq = synth_sequence(12, h, w, seed=0)
rec0 = O.intra_frame(seq[0], 16, 16, 4)["recon"]
import sys as _s
F = int(_s.argv[1])
rec = rec0
for f in range(1, F):
    rec = O.inter_frame(seq[f], [rec], 16, 16, 4)["recon"]
cur = seq[F].astype(np.int64); ref = rec.astype(np.int64)
c = np.zeros((h + 1, w + 1), np.int64); c[1:, 1:] = ref.cumsum(0).cumsum(1)
B4 = (c[4:, 4:] - c[:-4, 4:] - c[4:, :-4] + c[:-4, :-4]) >> 4
res = {k: [] for k in ("cur", "top4", "quad", "top16", "ideal")}
from numpy.lib.stride_tricks import sliding_window_view
win = sliding_window_view(ref, (16, 16))
for by in range(0, h // 16):
    for bx in range(0, w // 16):
        x, y = bx * 16, by * 16
        blk = cur[y:y+16, x:x+16]
        A = blk.reshape(4, 4, 4, 4).sum(axis=(1, 3)) >> 4
        lbs, sads, qs = [], [], []
        for dx in range(-16, 17):
            for dy in range(-16, 17):
                if not (0 <= x + dx < w - 16 and 0 <= y + dy < h - 16): continue
                dxi, di = dx + 16, dy + 16
                qs.append(((dxi >= 16) + 2 * (di >= 16)) if dxi < 32 else min(di // 16, 2))
                Bs = B4[y + dy: y + dy + 16: 4, x + dx: x + dx + 16: 4]
                lbs.append(16 * np.abs(A - Bs).sum() - 240)
                sads.append(np.abs(blk - win[y+dy, x+dx]).sum())
        lbs = np.array(lbs); sads = np.array(sads)
        order = np.argsort(lbs, kind="stable")
        qs = np.array(qs)
        qmins = [np.flatnonzero(qs == q)[np.argmin(lbs[qs == q])] for q in range(4) if (qs == q).any()]
        for k, U in (("cur", sads[order[0]]), ("top4", sads[order[:4]].min()), ("quad", sads[qmins].min()), ("top16", sads[order[:16]].min()), ("ideal", sads.min())):
            res[k].append(int((lbs <= U).sum()))
for k, v in res.items():
    v = np.array(v)
    print(f"{k:6s} blocks={len(v)} mean={v.mean():.1f} median={np.median(v):.0f} p90={np.percentile(v,90):.0f} frac>192={np.mean(v>192):.4f} frac>16={np.mean(v>16):.3f} frac==1={np.mean(v==1):.3f}")
