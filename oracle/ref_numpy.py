"""Faithful pure-Python/numpy restatement of the reference's per-block loops, used ONLY as
bench.py's CPU baseline ("kind": "port") and in tests as a checker.  TEST INFRASTRUCTURE.

It keeps the reference's cost structure on purpose: one np.mean(np.abs(a - b)) per
candidate in find_best_match (Encoder.py:678-717, 314-315), scipy.fftpack DCT/IDCT per
block (:779-817), np.round quantisation (:787), the Python RLE token loop (:1086-1131) and
per-block reconstruction (:824-932) — so its Mpx/s is what the reference achieves on the
same host (calibrated against the reference in the development container).
"""
from __future__ import annotations

import numpy as np
from scipy.fftpack import dct, idct


def _q_matrix(i, qp):
    q = np.zeros((i, i), dtype=int)
    for x in range(i):
        for y in range(i):
            q[x][y] = 2 ** qp if x + y < i - 1 else (2 ** (qp + 1) if x + y == i - 1 else 2 ** (qp + 2))
    return q


def _rle_len(block, n):
    result, flag, zero_count, nz = 0, 1, 0, 0
    for k in range(2 * n - 1):
        i, j = (0, k) if k < n else (k - n + 1, n - 1)
        while i < n and j >= 0:
            if block[i][j] != 0:
                if flag == 0:
                    if zero_count:
                        result += 1
                        zero_count = 0
                    nz = 0
                    flag = 1
                nz += 1
            else:
                if flag == 1:
                    if nz:
                        result += 1 + nz
                        nz = 0
                    zero_count = 0
                    flag = 0
                zero_count += 1
            i += 1
            j -= 1
    if nz:
        result += 1 + nz
    if zero_count:
        result += 1
    return result


def find_best_match(cur_block, ref, x, y, bs, sr):
    best_mae, best_mv = float("inf"), (0, 0, 0)
    h, w = ref.shape
    for dx in range(-sr, sr + 1):
        for dy in range(-sr, sr + 1):
            if 0 <= x + dx < w - bs and 0 <= y + dy < h - bs:
                mae = np.mean(np.abs(cur_block - ref[y + dy:y + dy + bs, x + dx:x + dx + bs]))
                if mae < best_mae:
                    best_mae, best_mv = mae, (dx, dy, 0)
                elif mae == best_mae:
                    if (abs(dx) + abs(dy), 0) < (abs(best_mv[0]) + abs(best_mv[1]), best_mv[2]):
                        best_mv = (dx, dy, 0)
    return best_mv, best_mae


def inter_rows(cur, ref, rows, bs=16, sr=16, qp=4):
    """P-frame work for the given block rows: ME, residual, DCT, quant, tokens, recon."""
    q = _q_matrix(bs, qp)
    h, w = ref.shape
    tokens = 0
    recon = np.zeros_like(ref)
    for by in rows:
        y = by * bs
        for x in range(0, cur.shape[1], bs):
            blk = cur[y:y + bs, x:x + bs]
            (dx, dy, _), _ = find_best_match(blk, ref, x, y, bs, sr)
            pred = ref[y + dy:y + dy + bs, x + dx:x + dx + bs]
            res = blk - pred
            tc = np.round(dct(dct(res, axis=0, norm="ortho"), axis=1, norm="ortho")).astype(int)
            qtc = np.round(tc / q).astype(int)
            tokens += _rle_len(qtc, bs)
            rb = np.round(idct(idct(qtc * q, axis=0, norm="ortho"), axis=1, norm="ortho")).astype(int)
            recon[y:y + bs, x:x + bs] = (pred + rb).astype(np.uint8)
    return tokens, recon


def intra_rows(cur, rows, bs=16, sr=16, qp=4):
    """I-frame work (mode 0) for the given block rows."""
    q = _q_matrix(bs, qp)
    h, w = cur.shape
    tokens = 0
    for by in rows:
        y = by * bs
        canvas = np.ones((bs, w)) * 128
        for x in range(0, w, bs):
            blk = cur[y:y + bs, x:x + bs]
            if x == 0:
                pred = np.ones((bs, bs)) * 128
            else:
                best_mae, best = float("inf"), 0
                for dx in range(-sr, sr + 1):
                    if x + dx >= 0 and x + dx + bs <= w:
                        mae = np.mean(np.abs(blk - canvas[:, x + dx:x + dx + bs]))
                        if mae < best_mae or (mae == best_mae and abs(dx) <= abs(best)):
                            best_mae, best = mae, dx
                pred = canvas[:, x + best:x + best + bs]
            res = blk - pred
            canvas[:, x:x + bs] = pred + res
            tc = np.round(dct(dct(res, axis=0, norm="ortho"), axis=1, norm="ortho")).astype(int)
            qtc = np.round(tc / q).astype(int)
            tokens += _rle_len(qtc, bs)
            np.round(idct(idct(qtc * q, axis=0, norm="ortho"), axis=1, norm="ortho")).astype(int)
    return tokens
