"""Offline analysis (test infrastructure: uses the C oracle).  Survivors of the plain run's
exact SEA bound (16 LBq - 240 <= U, the kernels' quantised 4x4 sums) per block of a whole 4K
P-frame F of the bench GOP (reference = the oracle's reconstruction chain), under choices of U:
  cur    the SAD of the smallest-bound candidate (what sea2_tile evaluates today);
  prev   min(cur, the SAD at the co-located block's motion vector in frame F-1);
  both   min(prev, the SAD at the left neighbour's vector in frame F);
  ideal  the block's minimum SAD (the floor any U can reach).
Prints the mean survivors, the mean 16-candidate passes (blocks with > 4 survivors:
ceil(n / 16); <= 4 and 1 take one partial pass / none) and the > 192 fraction.
Usage: python tests/analysis/sea_u_sources.py [F] [H]"""
import sys

import numpy as np

sys.path.insert(0, "/root/repo")
from numpy.lib.stride_tricks import sliding_window_view  # noqa: E402

from oracle import oracle as O  # noqa: E402
from streamoptima_amd.synth import synth_sequence  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 4
h = int(sys.argv[2]) if len(sys.argv) > 2 else 2160
w = 3840
seq = synth_sequence(F + 1, h, w, seed=0)
rec = O.intra_frame(seq[0], 16, 16, 4)["recon"]
prev = None
for f in range(1, F):
    r = O.inter_frame(seq[f], [rec], 16, 16, 4)
    rec, prev = r["recon"], r
cur_r = O.inter_frame(seq[F], [rec], 16, 16, 4)
cur = seq[F].astype(np.int32)
ref = rec.astype(np.int32)
nby, nbx = h // 16, w // 16
c = np.zeros((h + 1, w + 1), np.int64)
c[1:, 1:] = ref.cumsum(0).cumsum(1)
B4 = ((c[4:, 4:] - c[:-4, 4:] - c[4:, :-4] + c[:-4, :-4]) >> 4).astype(np.int32)   # [h-3, w-3]
A = (cur.reshape(nby, 4, 4, nbx, 4, 4).sum(axis=(2, 5)) >> 4).astype(np.int32)     # [nby, 4, nbx, 4]
ys, xs = np.arange(nby) * 16, np.arange(nbx) * 16
win = sliding_window_view(ref, (16, 16))


def sad_at(dx, dy):   # [nby, nbx] SAD at per-block offsets (0 where invalid)
    yy = np.clip(ys[:, None] + dy, 0, h - 16)
    xx = np.clip(xs[None, :] + dx, 0, w - 16)
    blk = cur.reshape(nby, 16, nbx, 16).transpose(0, 2, 1, 3)
    return np.abs(blk - win[yy, xx]).sum(axis=(2, 3))


lb = np.full((33, 33, nby, nbx), 1 << 30, np.int64)
for dxi in range(33):
    dx = dxi - 16
    vx = (xs + dx >= 0) & (xs + dx < w - 16)
    for di in range(33):
        dy = di - 16
        vy = (ys + dy >= 0) & (ys + dy < h - 16)
        yy = np.clip(ys + dy, 0, h - 16)
        xx = np.clip(xs + dx, 0, w - 16)
        Bs = B4[yy[:, None, None, None] + 4 * np.arange(4)[None, :, None, None],
                xx[None, None, :, None] + 4 * np.arange(4)[None, None, None, :]]   # [nby, 4, nbx, 4]
        v = np.abs(A - Bs).sum(axis=(1, 3))
        lb[dxi, di] = np.where(vy[:, None] & vx[None, :], v, 1 << 30)
flat = lb.reshape(33 * 33, nby, nbx)
k = flat.argmin(axis=0)                       # dx-major scan index, the kernel's tie order
U = {"cur": sad_at(k // 33 - 16, k % 33 - 16)}
mvp = prev["mv"][:, 0, :].reshape(nby, nbx, 3) if prev is not None else np.zeros((nby, nbx, 3), np.int16)
U["prev"] = np.minimum(U["cur"], sad_at(mvp[..., 0].astype(int), mvp[..., 1].astype(int)))
mvc = cur_r["mv"][:, 0, :].reshape(nby, nbx, 3)
left = np.zeros_like(mvc)
left[:, 1:] = mvc[:, :-1]
U["both"] = np.minimum(U["prev"], sad_at(left[..., 0].astype(int), left[..., 1].astype(int)))
U["ideal"] = cur_r["mae_num"].reshape(nby, nbx)
for name, u in U.items():
    n = ((16 * flat - 240) <= u[None]).sum(axis=0)
    passes = np.where(n > 4, -(-n // 16), 0)
    print(f"F={F} {name:6s} survivors mean {n.mean():7.2f} median {np.median(n):5.0f} p90 {np.percentile(n, 90):6.0f}"
          f"  n==1 {np.mean(n == 1):.3f}  n<=4 {np.mean(n <= 4):.3f}  passes/block {passes.mean():.3f}"
          f"  >192 {np.mean(n > 192):.4f}")
