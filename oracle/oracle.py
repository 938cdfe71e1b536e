"""ctypes binding of the C oracle (oracle/so_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker.  The product (streamoptima_amd) never imports this.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libso_oracle.so")

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = ctypes.CDLL(LIB_PATH)
        _lib.oc_sse_u8.restype = ctypes.c_int64
        _lib.oc_inter_frame.argtypes = None
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def dct1d(v: np.ndarray, inverse=False) -> np.ndarray:
    v = np.ascontiguousarray(v, dtype=np.float64).copy()
    n = v.shape[-1]
    f = lib().oc_dct3_1d if inverse else lib().oc_dct2_1d
    flat = v.reshape(-1, n)
    for row in flat:
        f(_p(row), ctypes.c_int(n))
    return v


def dct2d(block: np.ndarray, inverse=False) -> np.ndarray:
    n = block.shape[-1]
    a = np.ascontiguousarray(block, dtype=np.float64).reshape(-1, n, n)
    out = np.empty_like(a)
    f = lib().oc_idct2_2d if inverse else lib().oc_dct2_2d
    for i in range(a.shape[0]):
        f(_p(a[i]), _p(out[i]), ctypes.c_int(n))
    return out.reshape(block.shape)


def apply_2d_dct(res: np.ndarray) -> np.ndarray:
    n = res.shape[-1]
    a = np.ascontiguousarray(res, dtype=np.int32).reshape(-1, n, n)
    out = np.empty_like(a)
    for i in range(a.shape[0]):
        lib().oc_apply_2d_dct(_p(a[i]), _p(out[i]), ctypes.c_int(n))
    return out.reshape(res.shape)


def apply_2d_idct(deq: np.ndarray) -> np.ndarray:
    n = deq.shape[-1]
    a = np.ascontiguousarray(deq, dtype=np.int32).reshape(-1, n, n)
    out = np.empty_like(a)
    for i in range(a.shape[0]):
        lib().oc_apply_2d_idct(_p(a[i]), _p(out[i]), ctypes.c_int(n))
    return out.reshape(deq.shape)


def quantize(tc: np.ndarray, qp: int) -> np.ndarray:
    n = tc.shape[-1]
    a = np.ascontiguousarray(tc, dtype=np.int32)
    out = np.empty(a.shape, np.int16)
    lib().oc_quantize(_p(a), _p(out), ctypes.c_int(n), ctypes.c_int(qp))
    return out


def rle(q: np.ndarray) -> list:
    n = q.shape[-1]
    a = np.ascontiguousarray(q, dtype=np.int16)
    out = np.empty(2 * n * n + 2, np.int32)
    k = lib().oc_rle(_p(a), ctypes.c_int(n), _p(out))
    return out[:k].tolist()


def tokens(q: np.ndarray) -> int:
    n = q.shape[-1]
    a = np.ascontiguousarray(q, dtype=np.int16)
    return int(lib().oc_rle(_p(a), ctypes.c_int(n), None))


class FrameResult(dict):
    pass


def _refs_array(refs):
    arrs = [np.ascontiguousarray(r, dtype=np.uint8) for r in refs]
    ptrs = (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    return arrs, ptrs


def _i32(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.int32)


def inter_frame(cur: np.ndarray, refs, bs=16, sr=16, qp=4, qp_row=None, vbs=False,
                lam=0.015, me_mode=0, fme=False, fme_wrap=True, qp_map=None) -> FrameResult:
    """complete_inter_flow for one frame (oc_inter_frame_ex).  me_mode 0 = full search,
    1 = fast_me (serial predictor chain), 2 = fast_me under ParallelMode 2; fme = FMEEnable
    with the frac frame's uint8 wrap `fme_wrap` (True unless the reference list still holds
    the float64 start frame)."""
    cur = np.ascontiguousarray(cur, dtype=np.uint8)
    hp, wp = cur.shape
    h, w = refs[0].shape
    nb = (hp // bs) * (wp // bs)
    arrs, ptrs = _refs_array(refs)
    out = FrameResult(split=np.zeros(nb, np.uint8), mv=np.zeros((nb, 4, 3), np.int16),
                      qtc=np.zeros((nb, bs * bs), np.int16), tokens=np.zeros(nb, np.int32),
                      mae_num=np.zeros(nb, np.int64), recon=np.zeros((h, w), np.uint8))
    qr = None if qp_row is None else np.ascontiguousarray(qp_row, dtype=np.int32)
    qm = _i32(qp_map)
    rc = lib().oc_inter_frame_ex(_p(cur), hp, wp, ptrs, len(refs), h, w, bs, sr, qp,
                                 None if qr is None else _p(qr), None if qm is None else _p(qm), int(vbs),
                                 ctypes.c_double(lam),
                                 int(me_mode), int(bool(fme)), int(bool(fme_wrap)),
                                 _p(out["split"]), _p(out["mv"]), _p(out["qtc"]),
                                 _p(out["tokens"]), _p(out["mae_num"]), _p(out["recon"]))
    if rc != 0:
        raise ValueError(f"oc_inter_frame_ex failed: {rc}")
    return out


def fme_upsample(ref: np.ndarray, wrap=True) -> np.ndarray:
    """frac_me_reference_frame of one reference (oc_fme_upsample)."""
    ref = np.ascontiguousarray(ref, dtype=np.uint8)
    h, w = ref.shape
    out = np.zeros((2 * h - 1, 2 * w - 1), np.uint8)
    lib().oc_fme_upsample(_p(ref), h, w, int(bool(wrap)), _p(out))
    return out


def intra_frame(cur: np.ndarray, bs=16, sr=16, qp=6, qp_row=None, vbs=False,
                lam=0.015, qp_map=None) -> FrameResult:
    cur = np.ascontiguousarray(cur, dtype=np.uint8)
    hp, wp = cur.shape
    nb = (hp // bs) * (wp // bs)
    out = FrameResult(split=np.zeros(nb, np.uint8), mv=np.zeros((nb, 4), np.int16),
                      qtc=np.zeros((nb, bs * bs), np.int16), tokens=np.zeros(nb, np.int32),
                      mae_num=np.zeros(nb, np.int64), recon=np.zeros((hp, wp), np.uint8))
    qr = None if qp_row is None else np.ascontiguousarray(qp_row, dtype=np.int32)
    qm = _i32(qp_map)
    rc = lib().oc_intra_frame_ex(_p(cur), hp, wp, bs, sr, qp, None if qr is None else _p(qr),
                                 None if qm is None else _p(qm), int(vbs), ctypes.c_double(lam), _p(out["split"]), _p(out["mv"]),
                              _p(out["qtc"]), _p(out["tokens"]), _p(out["mae_num"]),
                              _p(out["recon"]))
    if rc != 0:
        raise ValueError(f"oc_intra_frame failed: {rc}")
    return out


def inter_recon(refs, split, mv, qtc, bs=16, qp=4, qp_row=None, fme=False, fme_wrap=True,
                qp_map=None) -> np.ndarray:
    h, w = refs[0].shape
    arrs, ptrs = _refs_array(refs)
    recon = np.zeros((h, w), np.uint8)
    qr = None if qp_row is None else np.ascontiguousarray(qp_row, dtype=np.int32)
    qm = _i32(qp_map)
    lib().oc_inter_recon_ex(ptrs, len(refs), h, w, bs, qp, None if qr is None else _p(qr),
                            None if qm is None else _p(qm), int(bool(fme)),
                            int(bool(fme_wrap)), _p(np.ascontiguousarray(split, np.uint8)),
                            _p(np.ascontiguousarray(mv, np.int16)),
                            _p(np.ascontiguousarray(qtc, np.int16)), _p(recon))
    return recon


def qp_map(tokens, nbx, nby, qp_rd, qp_row=None, roi=None, qp_lo=0, qp_hi=12) -> np.ndarray:
    """Per-block QP map of ROI / two-pass RC (oc_qp_map); tokens/roi flat [nby*nbx] or None."""
    out = np.zeros(nbx * nby, np.int32)
    t, r, qr = _i32(tokens), _i32(roi), _i32(qp_row)
    lib().oc_qp_map(None if t is None else _p(t), nbx, nby, qp_rd, None if qr is None else _p(qr),
                    None if r is None else _p(r), qp_lo, qp_hi, _p(out))
    return out


def sse(a: np.ndarray, b: np.ndarray) -> int:
    a = np.ascontiguousarray(a, np.uint8)
    b = np.ascontiguousarray(b, np.uint8)
    return int(lib().oc_sse_u8(_p(a), _p(b), ctypes.c_int64(a.size)))


def me_block(cur: np.ndarray, refs, x: int, y: int, bs: int, sr: int) -> tuple:
    cur = np.ascontiguousarray(cur, dtype=np.uint8)
    h, w = refs[0].shape
    arrs, ptrs = _refs_array(refs)
    out = np.zeros(4, np.int32)
    lib().oc_me_block(_p(cur), cur.shape[1], ptrs, len(refs), h, w, x, y, bs, sr, _p(out))
    return tuple(int(v) for v in out)
