"""Test helper: a plain-Python writer of the packed symbol stream (so_pack.hip's format), the
checker for so_pack_frames.  Per block: split, mv values, then each (sub-)block's RLE token
list produced by the reference's own loop (entropy_encoder_block, Encoder.py:1086-1131,
restated with its flag / run variables), every number a zigzag LEB128 varint."""
import numpy as np


def rle_reference_loop(block: np.ndarray, n: int) -> list:
    res, vals, nzc, zc, flag = [], [], 0, 0, 1
    for k in range(2 * n - 1):
        i, j = (0, k) if k < n else (k - n + 1, n - 1)
        while i < n and j >= 0:
            x = int(block[i, j])
            if x != 0:
                if flag == 0:
                    if zc:
                        res.append(zc)
                        zc = 0
                    vals, nzc, flag = [], 0, 1
                vals.append(x)
                nzc += 1
            else:
                if flag == 1:
                    if nzc:
                        res.append(-nzc)
                        res.extend(vals)
                        vals, nzc = [], 0
                    zc, flag = 0, 0
                zc += 1
            i, j = i + 1, j - 1
    if nzc:
        res.append(-nzc)
        res.extend(vals)
    if zc:
        res.append(0)
    return res


def varint(v: int) -> bytes:
    z = 2 * v if v >= 0 else -2 * v - 1
    out = bytearray()
    while True:
        b = z & 0x7F
        z >>= 7
        out.append(b | (0x80 if z else 0))
        if not z:
            return bytes(out)


def pack_frame(split, mv, qtc, bs: int, frame_type: int) -> bytes:
    split, mv, qtc = np.asarray(split), np.asarray(mv), np.asarray(qtc)
    sb = bs // 2
    out = bytearray()
    for b in range(split.size):
        sp = int(split[b])
        nums = [sp]
        for j in range(4 if sp else 1):
            nums.extend(int(x) for x in (mv[b, j] if frame_type == 1 else [mv[b, j]]))
        if sp:
            for j in range(4):
                nums.extend(rle_reference_loop(qtc[b, j * sb * sb:(j + 1) * sb * sb].reshape(sb, sb), sb))
        else:
            nums.extend(rle_reference_loop(qtc[b].reshape(bs, bs), bs))
        for x in nums:
            out += varint(x)
    return bytes(out)


def random_symbols(rng, nb: int, bs: int, frame_type: int, vbs: bool):
    """Symbols with the shapes the kernels write: sparse small coefficients, some dense
    blocks, int16 extremes, all-zero blocks, split blocks when vbs."""
    split = (rng.random(nb) < 0.4).astype(np.uint8) if vbs else np.zeros(nb, np.uint8)
    mv = rng.integers(-16, 17, size=(nb, 4, 3) if frame_type == 1 else (nb, 4)).astype(np.int16)
    if frame_type == 1:
        mv[..., 2] = 0
    qtc = np.zeros((nb, bs * bs), np.int16)
    for b in range(nb):
        kind = b % 5
        if kind == 1:
            m = rng.random(bs * bs) < 0.15
            qtc[b, m] = rng.integers(-70, 71, size=int(m.sum()))
        elif kind == 2:
            qtc[b] = rng.integers(-300, 301, size=bs * bs)
        elif kind == 3:
            qtc[b, :4] = [32767, -32768, 1, -1]
            qtc[b, -1] = 5
        elif kind == 4:
            qtc[b, 0] = rng.integers(-3, 4)
    return split, mv, qtc
