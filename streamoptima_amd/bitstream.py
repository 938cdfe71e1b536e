"""Text bitstream of the reference (host-side formatting of the GPU symbols).

  * entropy_encoder_block   — Encoder.py:1086-1131: anti-diagonal scan, RLE tokens
                              (-count, values... for non-zero runs, count for zero runs,
                              a trailing zero run as a single 0).  Values keep the input's
                              element type (np.int64 for the package arrays), so str()
                              of the list matches the reference byte for byte.
  * differential_encoder_frame — Encoder.py:1419-1520 (MV / QP differential line,
                              including the reference's split-under-RC intra quirk).
  * entropy_encoder_frame   — Encoder.py:1522-1542.
  * varints / unpack_frame  — host decoder of the packed symbol stream the GPU writes
                              (so_pack_frames, include/streamoptima.h; format in so_pack.hip).
"""
from __future__ import annotations

import ast
import re
from functools import lru_cache

import numpy as np


@lru_cache(maxsize=8)
def scan_order(n: int) -> np.ndarray:
    """flat indices i*n+j in the order entropy_encoder_block visits them."""
    order = []
    for k in range(2 * n - 1):
        i, j = (0, k) if k < n else (k - n + 1, n - 1)
        while i < n and j >= 0:
            order.append(i * n + j)
            i += 1
            j -= 1
    return np.array(order, dtype=np.int64)


def entropy_encoder_block(residual_block, block_size) -> list:
    arr = np.asarray(residual_block)
    vals = arr.reshape(-1)[scan_order(block_size)] if arr.ndim == 2 else arr.reshape(-1)
    nz = vals != 0
    out = []
    n = len(vals)
    if n == 0:
        return out
    # boundaries of maximal runs
    change = np.flatnonzero(nz[1:] != nz[:-1]) + 1
    starts = np.concatenate(([0], change))
    ends = np.concatenate((change, [n]))
    for s, e in zip(starts.tolist(), ends.tolist()):
        if nz[s]:
            out.append(-(e - s))
            out.extend(vals[s:e])      # numpy scalars, like residual_block[i][j]
        elif e == n:
            out.append(0)
        else:
            out.append(e - s)
    return out


def token_count(residual_block, block_size) -> int:
    vals = np.asarray(residual_block).reshape(-1)
    nz = vals != 0
    return int(nz.sum() + 1 + (nz[1:] != nz[:-1]).sum()) if vals.size else 0


def differential_encoder_frame(frame_type, mv_for_frame, Qp_for_frame, rc_flag, num_blocks_per_row) -> str:
    rc = rc_flag is not None and rc_flag > 0
    parts = []
    ref_qp = 0
    diff_qp = None
    if frame_type == 0:
        ref = 0
        for j, mv in enumerate(mv_for_frame):
            rc_row = rc and j % num_blocks_per_row == 0
            if rc_row:
                diff_qp = Qp_for_frame[int(j // num_blocks_per_row)] - ref_qp
            if mv[0] == 0:
                d = mv[1] - ref
                s = (f"{diff_qp}@0'({d})" if rc_row else f"0'({d})")
                parts.append(s if j == 0 else ";" + s)
                ref = mv[1]
            else:
                for k, sb in enumerate(mv[1]):
                    d = sb - ref
                    if k == 0:
                        parts.append(f";{d}@1'({d}," if rc_row else f";1'({d},")
                    elif k == 3:
                        parts.append(f"{d})")
                    else:
                        parts.append(f"{d},")
                    ref = sb
            if rc_row:
                ref_qp = Qp_for_frame[int(j // num_blocks_per_row)]
    else:
        ref = (0, 0, 0)
        for j, mv in enumerate(mv_for_frame):
            rc_row = rc and j % num_blocks_per_row == 0
            if rc_row:
                diff_qp = Qp_for_frame[int(j // num_blocks_per_row)] - ref_qp
            if mv[0] == 0:
                m = mv[1]
                d = (m[0] - ref[0], m[1] - ref[1], m[2] - ref[2])
                s = (f"{diff_qp}@0'{d}" if rc_row else f"0'{d}")
                parts.append(s if j == 0 else ";" + s)
                ref = m
            else:
                for k, sb in enumerate(mv[1]):
                    d = (sb[0] - ref[0], sb[1] - ref[1], sb[2] - ref[2])
                    if k == 0:
                        parts.append(f";{diff_qp}@1'({d}," if rc_row else f";1'({d},")
                    elif k == 3:
                        parts.append(f"{d})")
                    else:
                        parts.append(f"{d},")
                    ref = sb
            if rc_row:
                ref_qp = Qp_for_frame[int(j // num_blocks_per_row)]
    return "".join(parts)


def entropy_encoder_frame(frame_residuals, block_size) -> str:
    parts = []
    for i, residual in enumerate(frame_residuals):
        if residual[0] == 0:
            s = "0'(" + str(entropy_encoder_block(residual[1], block_size)) + ")"
            parts.append(s if i == 0 else ";" + s)
        else:
            for k, sb in enumerate(residual[1]):
                t = str(entropy_encoder_block(sb, block_size // 2))
                if k == 0:
                    parts.append(";1'(" + t + ",")
                elif k == 3:
                    parts.append(t + ")")
                else:
                    parts.append(t + ",")
    return "".join(parts)


# ---- parsers (decoder.py:547-690) ------------------------------------------------------------
# The reference parses with eval(); the tokens are int / tuple / list literals -- numpy 2
# prints the package's values as np.int64(v) -- so unwrapping those and ast.literal_eval
# read exactly the same values without executing anything.
_NP_SCALAR = re.compile(r"np\.u?int(?:8|16|32|64)\((-?\d+)\)")


def _literal(text: str):
    return ast.literal_eval(_NP_SCALAR.sub(r"\1", text))

def entropy_decoder_block(encoded_block, block_size) -> list:
    """decoder.py:547-586: RLE tokens -> block_size x block_size list of lists (anti-diagonal
    scan; a zero token ends the block, trailing positions stay 0)."""
    arr = []
    i = 0
    while i < len(encoded_block):
        t = encoded_block[i]
        if t < 0:
            arr.extend(encoded_block[i + 1:i + 1 - t])
            i += -t
        else:
            if t == 0:
                break
            arr.extend([0] * t)
        i += 1
    out = np.zeros(block_size * block_size, dtype=int)
    order = scan_order(block_size)
    m = min(len(arr), len(order))
    out[order[:m]] = arr[:m]
    return out.reshape(block_size, block_size).tolist()


def differential_decoder_frame(line: str, rc_flag, num_blocks_per_row):
    """decoder.py:589-644: '<type>|...' -> (frame_type, per-block mvs, per-row QPs)."""
    rc = rc_flag is not None and rc_flag > 0
    raw = line.strip().split("|")
    frame_type = int(raw[0])
    mvs, qps = [], []
    ref_qp = 0
    ref = 0 if frame_type == 0 else (0, 0, 0)
    for j, tok in enumerate(raw[1].split(";")):
        if rc and j % num_blocks_per_row == 0:
            q, tok = tok.split("@")
            ref_qp = ref_qp + int(_literal(q))
            qps.append(ref_qp)
        split, body = tok.split("'")
        v = _literal(body)
        if frame_type == 0:
            if split == "0":
                ref = ref + int(v)
                mvs.append((0, ref))
            else:
                sub = []
                for d in v:
                    ref = ref + d
                    sub.append(ref)
                mvs.append((1, sub))
        else:
            if split == "0":
                ref = (ref[0] + v[0], ref[1] + v[1], ref[2] + v[2])
                mvs.append((0, ref))
            else:
                sub = []
                for d in v:
                    ref = (ref[0] + d[0], ref[1] + d[1], ref[2] + d[2])
                    sub.append(ref)
                mvs.append((1, sub))
    return frame_type, mvs, qps


def entropy_decoder_frame(line: str, block_size) -> list:
    """decoder.py:646-664: residual RLE line -> [(0, QTC) | (1, [QTC x 4])]."""
    out = []
    for tok in line.strip().split(";"):
        split, body = tok.split("'")
        v = _literal(body)
        if split == "0":
            out.append((0, np.array(entropy_decoder_block(v, block_size))))
        else:
            out.append((1, [np.array(entropy_decoder_block(sb, block_size // 2)) for sb in v]))
    return out


# ---- packed symbol stream (so_pack_frames) -----------------------------------------------------
def varints(buf) -> np.ndarray:
    """Zigzag LEB128 varints -> int64 values (vectorised over the whole stream)."""
    b = np.asarray(buf, dtype=np.uint8).reshape(-1)
    if b.size == 0:
        return np.zeros(0, dtype=np.int64)
    ends = np.flatnonzero((b & 0x80) == 0)
    if ends.size == 0 or ends[-1] != b.size - 1:
        raise ValueError("packed stream ends inside a varint")
    starts = np.concatenate(([0], ends[:-1] + 1))
    lens = ends - starts + 1
    z = np.zeros(ends.size, dtype=np.int64)
    for k in range(int(lens.max())):
        m = lens > k
        z[m] |= (b[starts[m] + k].astype(np.int64) & 0x7F) << (7 * k)
    return (z >> 1) ^ -(z & 1)


def unpack_frame(buf, nb: int, bs: int, frame_type: int) -> dict:
    """One frame's packed stream -> {"split", "mv", "qtc"} in the canonical symbol layout
    (mv entries past the first of an unsplit block stay 0)."""
    v = varints(buf).tolist()
    inter = frame_type == 1
    split = np.zeros(nb, dtype=np.uint8)
    mv = np.zeros((nb, 4, 3) if inter else (nb, 4), dtype=np.int16)
    qtc = np.zeros((nb, bs * bs), dtype=np.int16)
    sb = bs // 2
    p = 0
    try:
        for b in range(nb):
            sp = v[p]
            p += 1
            split[b] = sp
            for j in range(4 if sp else 1):
                if inter:
                    mv[b, j] = v[p:p + 3]
                    p += 3
                else:
                    mv[b, j] = v[p]
                    p += 1
            for n, off in ([(sb, j * sb * sb) for j in range(4)] if sp else [(bs, 0)]):
                order, k = scan_order(n), 0
                while k < n * n:
                    t = v[p]
                    p += 1
                    if t < 0:
                        qtc[b, off + order[k:k - t]] = v[p:p - t]
                        p, k = p - t, k - t
                    elif t == 0:
                        break
                    else:
                        k += t
    except IndexError:
        raise ValueError(f"packed stream ends inside block {b}") from None
    if p != len(v):
        raise ValueError(f"{len(v) - p} values after the last block")
    return {"split": split, "mv": mv, "qtc": qtc}


# ---- per-block QP map line (build extension: ROI / two-pass RC) --------------------------------
def qp_map_line(qp_map, qp_rows, base_qp, num_blocks_per_row) -> str:
    """Per-block QPs as comma-separated deltas against the row's QP (the per-row QP the
    reference line already carries, or the frame QP without rate control)."""
    nbx = int(num_blocks_per_row)
    q = np.asarray(qp_map).reshape(-1, nbx)
    base = np.asarray(qp_rows if qp_rows else [base_qp] * q.shape[0]).reshape(-1, 1)
    return ",".join(str(int(v)) for v in (q - base).reshape(-1))


def parse_qp_map_line(line: str, qp_rows, base_qp, num_blocks_per_row) -> np.ndarray:
    nbx = int(num_blocks_per_row)
    d = np.array([int(t) for t in line.strip().split(",")], np.int32).reshape(-1, nbx)
    base = np.asarray(qp_rows if qp_rows else [base_qp] * d.shape[0], np.int32).reshape(-1, 1)
    return (d + base).reshape(-1).astype(np.int32)
