"""Host materialisation of the reference's `encoded_package` (Encoder.py:1877-1892).

The GPU path keeps symbols as flat device arrays; the reference's package is lists of
per-block tuples holding numpy int64 arrays, which costs tens of milliseconds per 4K
frame to build in Python.  LazyPackage builds each entry the first time it is read.
"""
from __future__ import annotations

import numpy as np

from .engine import FrameSymbols


def symbols_to_host(sym: FrameSymbols) -> dict:
    return {"frame_type": sym.frame_type,
            "split": sym.split.cpu().numpy(),
            "mv": sym.mv.cpu().numpy(),
            "qtc": sym.qtc.cpu().numpy(),
            "tokens": sym.tokens.cpu().numpy(),
            "mae_num": sym.mae_num.cpu().numpy(),
            "recon": sym.recon.cpu().numpy()}


def frame_mvs(host: dict, bs: int) -> list:
    """inter: [(0, (dx, dy, ref)) | (1, [(dx, dy, ref) x 4])]; intra: [(0, dx) | (1, [dx x 4])]
    (inter_prediction :569-578, intra_prediction :1317-1327)."""
    split = host["split"].tolist()
    mv = host["mv"].tolist()
    out = []
    if host["frame_type"] == 1:
        for s, m in zip(split, mv):
            if s:
                out.append((1, [tuple(m[0]), tuple(m[1]), tuple(m[2]), tuple(m[3])]))
            else:
                out.append((0, tuple(m[0])))
    else:
        for s, m in zip(split, mv):
            out.append((1, list(m)) if s else (0, m[0]))
    return out


def frame_residuals(host: dict, bs: int) -> list:
    """[(0, QTC int64 bs x bs) | (1, [QTC sub x 4])] (complete_*_flow :1611-1625, :1680-1694)."""
    split = host["split"]
    q = host["qtc"].astype(np.int64)
    sb = bs // 2
    full = q.reshape(-1, bs, bs)
    sub = q.reshape(-1, 4, sb, sb)
    out = []
    for i, s in enumerate(split.tolist()):
        if s:
            out.append((1, [sub[i, 0], sub[i, 1], sub[i, 2], sub[i, 3]]))
        else:
            out.append((0, full[i]))
    return out


class LazyPackage(dict):
    """dict with the reference's keys; heavy entries are built on first access."""

    _LAZY = ("MVS per Frame", "approx residual", "MAE per Frame")

    def __init__(self, codec, symbols, psnr, frame_types, qp_rows):
        super().__init__()
        self._codec = codec
        self._symbols = symbols
        self._host = None
        self["block size"] = codec.block_size
        self["num frames"] = codec.frames
        self["height in pixels"] = codec.h_pixels
        self["width in pixels"] = codec.w_pixels
        self["search range"] = codec.search_range
        self["PSNR per frame"] = psnr
        self["SSIM per frame"] = [float("nan")] * len(psnr)   # skimage SSIM is out of scope
        self["Qp_per_row_per_frame"] = qp_rows
        self["frame_type_seq"] = list(frame_types)

    def _hosts(self):
        if self._host is None:
            self._host = [symbols_to_host(s) for s in self._symbols]
        return self._host

    def _build(self, key):
        bs = self._codec.block_size
        if key == "MVS per Frame":
            return [frame_mvs(h, bs) for h in self._hosts()]
        if key == "approx residual":
            return [frame_residuals(h, bs) for h in self._hosts()]
        if key == "MAE per Frame":
            return [self._codec._avg_mae(h["mae_num"]) for h in self._hosts()]
        raise KeyError(key)

    def __missing__(self, key):
        if key in self._LAZY:
            v = self._build(key)
            self[key] = v
            return v
        raise KeyError(key)

    def __contains__(self, key):
        return key in self._LAZY or super().__contains__(key)

    def keys(self):
        return list(super().keys()) + [k for k in self._LAZY if not super().__contains__(k)]

    def any(self):  # the reference calls encoded_package.any() (Encoder.py:1004)
        return True
