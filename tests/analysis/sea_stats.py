"""Offline analysis (test infrastructure: uses the C oracle, so it lives under tests/).
Offline survivor statistics of the exact SEA pruning in me_sea2_kernel (so_me.hip) on the
bench content: per block, count the candidates whose 4x4-sum lower bound does not exceed the
SAD of the smallest-bound candidate.  Uses the C oracle for the I-frame reconstruction."""
import numpy as np, sys
sys.path.insert(0, "/root/repo")
from streamoptima_amd.synth import synth_sequence
from oracle import oracle as O
h, w = 272, 480
seq = synth_sequence(3, h, w, seed=1)
# ref variants: original frame 0, and the oracle reconstruction of frame 0 (I-frame QP4)
rec0 = O.intra_frame(seq[0], 16, 16, 4)["recon"]
def stats(cur, ref, label):
    cur = cur.astype(np.int64); ref = ref.astype(np.int64)
    # 4x4 box sums of ref at every position
    c = np.zeros((h + 1, w + 1), np.int64); c[1:, 1:] = ref.cumsum(0).cumsum(1)
    B4 = c[4:, 4:] - c[:-4, 4:] - c[4:, :-4] + c[:-4, :-4]   # B4[y, x] = sum ref[y:y+4, x:x+4]
    nsurv = []
    for by in range(1, h // 16 - 1):
        for bx in range(1, w // 16 - 1):
            x, y = bx * 16, by * 16
            blk = cur[y:y+16, x:x+16]
            A = blk.reshape(4, 4, 4, 4).sum(axis=(1, 3))   # [j, i]
            lbs, sads = [], []
            for dx in range(-16, 17):
                for dy in range(-16, 17):
                    if not (0 <= x + dx < w - 16 and 0 <= y + dy < h - 16):
                        continue
                    Bs = B4[y + dy: y + dy + 16: 4, x + dx: x + dx + 16: 4]
                    lbs.append(np.abs(A - Bs).sum())
                    sads.append(np.abs(blk - ref[y+dy:y+dy+16, x+dx:x+dx+16]).sum())
            lbs = np.array(lbs); sads = np.array(sads)
            U = sads[np.argmin(lbs)]
            nsurv.append(int((lbs <= U).sum()))
    nsurv = np.array(nsurv)
    print(f"{label}: blocks={len(nsurv)} survivors mean={nsurv.mean():.1f} median={np.median(nsurv):.0f} p90={np.percentile(nsurv,90):.0f} max={nsurv.max()} frac>192={np.mean(nsurv>192):.3f} frac>64={np.mean(nsurv>64):.3f}")
stats(seq[1], seq[0], "ref=original")
stats(seq[1], rec0, "ref=recon(I,QP4)")
