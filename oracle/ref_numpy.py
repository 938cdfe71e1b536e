"""Faithful pure-Python/numpy restatement of the reference's per-block loops, used ONLY as
bench.py's CPU baseline ("kind": "port") and in tests as a checker.  TEST INFRASTRUCTURE.

It keeps the reference's cost structure on purpose, call for call:
  * find_best_match (Encoder.py:678-717): refs outer, dx, dy; one bound test, one
    self.compute_mae = np.mean(np.abs(a - b)) (:314-315) per candidate and
    self.is_better_mv (:771-773) on ties -- as bound-method calls, like the reference's;
  * apply_2d_dct / quantize_TC / rescale_QTC / apply_2d_idct (:779-821) with scipy.fftpack;
  * entropy_encoder_block (:1086-1131) building the token LIST (appends / extends), whose
    len() is the block's token count, as complete_inter_flow does (:1683);
  * reconstruct_block (:824-827) per block;
  * intra (mode 0, :1010-1045, :1238-1347): an H x W float canvas of 128s per frame (the
    reference's hard-coded 288 x 352 generalised), search over
    canvas rows, canvas written back with pred + residual.
Its Mpx/s is what the reference achieves on the same host; oracle/calibrate_cpu_port.py
times both on identical 4K rows in the development container.
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


class PortCodec:
    """The per-block methods the reference's frame flows call, with the same shapes."""

    def __init__(self, bs=16, sr=16, qp=4):
        self.block_size, self.search_range = bs, sr
        self.Q = _q_matrix(bs, qp)

    # Encoder.py:314-315
    def compute_mae(self, block1, block2):
        return np.mean(np.abs(block1 - block2))

    # Encoder.py:771-773
    def is_better_mv(self, mv1, mv2):
        return (abs(mv2[0]) + abs(mv2[1]), mv2[2]) < (abs(mv1[0]) + abs(mv1[1]), mv1[2])

    # Encoder.py:678-717 (FMEEnable off)
    def find_best_match(self, current_block, ref_frames, x, y, block_size, search_range):
        best_mae = float("inf")
        best_mv = (0, 0, 0)
        for ref_idx, ref_frame in enumerate(ref_frames):
            for dx in range(-search_range, search_range + 1):
                for dy in range(-search_range, search_range + 1):
                    if 0 <= x + dx < ref_frame.shape[1] - block_size and 0 <= y + dy < ref_frame.shape[0] - block_size:
                        ref_block = ref_frame[y + dy:y + dy + block_size, x + dx:x + dx + block_size]
                        mae = self.compute_mae(current_block, ref_block)
                        if mae < best_mae:
                            best_mae = mae
                            best_mv = (dx, dy, ref_idx)
                        elif mae == best_mae:
                            if self.is_better_mv(best_mv, (dx, dy, ref_idx)):
                                best_mv = (dx, dy, ref_idx)
        return best_mv, best_mae

    # Encoder.py:779-789, 810-821
    def apply_2d_dct(self, input_block):
        return np.round(dct(dct(input_block, axis=0, norm="ortho"), axis=1, norm="ortho")).astype(int)

    def quantize_TC(self, TC, Q):
        return np.round(TC / Q).astype(int)

    def rescale_QTC(self, QTC, Q):
        return QTC * Q

    def apply_2d_idct(self, input_block):
        return np.round(idct(idct(input_block, axis=0, norm="ortho"), axis=1, norm="ortho")).astype(int)

    # Encoder.py:824-827
    def reconstruct_block(self, predicted_block, residual_block):
        return (predicted_block + residual_block).astype(np.uint8)

    # Encoder.py:1086-1131: the token list (anti-diagonal RLE)
    def entropy_encoder_block(self, residual_block, block_size):
        n = block_size
        result, non_zero_values = [], []
        flag, zero_count, non_zero_count = 1, 0, 0
        for k in range(2 * n - 1):
            i, j = (0, k) if k < n else (k - n + 1, n - 1)
            while i < n and j >= 0:
                if residual_block[i][j] != 0:
                    if flag == 0:
                        if zero_count:
                            result.append(zero_count)
                            zero_count = 0
                        non_zero_values = []
                        non_zero_count = 0
                        flag = 1
                    non_zero_values.append(residual_block[i][j])
                    non_zero_count += 1
                else:
                    if flag == 1:
                        if non_zero_count:
                            result.append(-non_zero_count)
                            result.extend(non_zero_values)
                            non_zero_values = []
                            non_zero_count = 0
                        zero_count = 0
                        flag = 0
                    zero_count += 1
                i += 1
                j -= 1
        if non_zero_count:
            result.append(-non_zero_count)
            result.extend(non_zero_values)
        if zero_count:
            result.extend([0])
        return result


def _rle_len(block, n):
    return len(PortCodec(n).entropy_encoder_block(block, n))


def find_best_match(cur_block, ref, x, y, bs, sr):
    return PortCodec(bs, sr).find_best_match(cur_block, [ref], x, y, bs, sr)


def inter_rows(cur, ref, rows, bs=16, sr=16, qp=4):
    """P-frame work for the given block rows (complete_inter_flow's per-block work,
    Encoder.py:462-585, 1665-1697, 831-932): ME, residual, DCT, quant, token list, recon."""
    c = PortCodec(bs, sr, qp)
    refs = [ref]
    tokens = 0
    recon = np.zeros_like(ref)
    for by in rows:
        y = by * bs
        for x in range(0, cur.shape[1], bs):
            blk = cur[y:y + bs, x:x + bs]
            (dx, dy, r), _ = c.find_best_match(blk, refs, x, y, bs, sr)
            pred = refs[r][y + dy:y + dy + bs, x + dx:x + dx + bs]
            res = blk - pred
            qtc = c.quantize_TC(c.apply_2d_dct(res), c.Q)
            tokens += len(c.entropy_encoder_block(qtc, bs))
            rb = c.apply_2d_idct(c.rescale_QTC(qtc, c.Q))
            recon[y:y + bs, x:x + bs] = c.reconstruct_block(pred, rb)
    return tokens, recon


def intra_rows(cur, rows, bs=16, sr=16, qp=4):
    """I-frame work (mode 0, Encoder.py:1010-1045, 1238-1347) for the given block rows on
    an H x W canvas of 128s."""
    c = PortCodec(bs, sr, qp)
    h, w = cur.shape
    tokens = 0
    canvas = np.ones((h, w)) * 128
    for by in rows:
        y = by * bs
        for x in range(0, w, bs):
            blk = cur[y:y + bs, x:x + bs]
            if x == 0:
                pred = np.ones((bs, bs)) * 128
                c.compute_mae(blk, pred)
            else:
                best_mae, best = float("inf"), 0
                for dx in range(-sr, sr + 1):
                    if x + dx >= 0 and x + dx + bs <= canvas.shape[1]:
                        ref_block = canvas[y:y + bs, x + dx:x + dx + bs]
                        mae = c.compute_mae(blk, ref_block)
                        if mae < best_mae:
                            best_mae, best = mae, dx
                        elif mae == best_mae:
                            if abs(dx) < abs(best) or abs(dx) == abs(best):
                                best = dx
                pred = canvas[y:y + bs, x + best:x + best + bs]
            res = blk - pred
            canvas[y:y + bs, x:x + bs] = pred + res
            qtc = c.quantize_TC(c.apply_2d_dct(res), c.Q)
            tokens += len(c.entropy_encoder_block(qtc, bs))
            c.apply_2d_idct(c.rescale_QTC(qtc, c.Q))
    return tokens


def _pool_inter(args):
    """One block row of inter_rows in a worker (the ParallelMode-2 analogue: the task carries
    only the rows its search window touches, not whole frames)."""
    cur_band, ref_band, local_row, bs, sr, qp = args
    return inter_rows(cur_band, ref_band, [local_row], bs, sr, qp)[0]


def inter_rows_pool(cur, ref, rows, procs, bs=16, sr=16, qp=4):
    """inter_rows over `procs` worker processes, one block row per task (Encoder.py:477-499
    ParallelMode 2 dispatches blocks to Pool(8); here the unit is a row of blocks and each
    task carries the +-sr band of the reference it searches)."""
    from multiprocessing import get_context
    h = ref.shape[0]
    if sr % bs:
        raise ValueError("search range must be a multiple of the block size for banded tasks")
    tasks = []
    for by in rows:
        # the band holds every row the block's candidates read, plus one more below so the
        # strict bound y + dy < H - bs admits exactly the full frame's candidates (a band
        # clipped at the frame's own top or bottom keeps the true edge)
        y0 = max(0, by * bs - sr)
        y1 = min(h, by * bs + bs + sr + 1)
        tasks.append((cur[y0:y1].copy(), ref[y0:y1].copy(), (by * bs - y0) // bs, bs, sr, qp))
    with get_context("fork").Pool(procs) as pool:
        return sum(pool.map(_pool_inter, tasks))
