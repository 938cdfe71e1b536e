"""A binary container for the packed symbol stream (so_pack_frames) -- the compact counterpart of
the reference's two text files (transmit_bitstream, Encoder.py:1544-1573; decode_bitstream,
decoder.py:686-709).

    header   b"SOPK" | u32 version 1 | u32 H | u32 W | u32 bs | u32 nframes | u32 nb
    frame    u8 frame_type | u16 nqp | i8 qp[nqp] (per-row QPs under rate control, else 0)
             | u32 nbytes | u16 block_bytes[nb] | bytes[nbytes]

Little endian.  block_bytes lets the GPU decoder (so_unpack_frames) start every block in
parallel: the offsets are their exclusive prefix sums.  Per-block QP maps (ROI / two-pass RC)
are not carried: such GOPs use the text bitstream.
"""
from __future__ import annotations

import struct

import numpy as np
import torch

MAGIC, VERSION = b"SOPK", 1


def write(path: str, eng, symbols: list, qp_rows: list | None = None) -> int:
    """Pack `symbols` (FrameSymbols on the device) and write the container; returns its size."""
    if any(s.extra.get("qp_map") is not None for s in symbols):
        raise NotImplementedError("per-block QP maps (ROI / two-pass RC) are not carried by the packed container")
    offs, out = eng.pack_symbols(symbols)
    offs_h = offs.cpu().numpy().astype(np.int64)
    size = 0
    with open(path, "wb") as f:
        hdr = MAGIC + struct.pack("<6I", VERSION, eng.h, eng.w, eng.bs, len(symbols), eng.nb)
        f.write(hdr)
        size += len(hdr)
        for i, s in enumerate(symbols):
            q = list(qp_rows[i]) if qp_rows and qp_rows[i] else []
            nbytes = int(offs_h[i, -1])
            lens = np.diff(offs_h[i]).astype(np.uint16)
            rec = (struct.pack("<BH", int(s.frame_type), len(q)) + np.asarray(q, np.int8).tobytes()
                   + struct.pack("<I", nbytes) + lens.tobytes() + out[i, :nbytes].cpu().numpy().tobytes())
            f.write(rec)
            size += len(rec)
    return size


def read(path: str, device) -> dict:
    """-> {"h", "w", "bs", "nb", "frame_types", "qp_rows", "packed": [device uint8],
    "offs": [device int32 [nb + 1]]}."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != MAGIC:
        raise ValueError(f"{path}: not a packed StreamOptima bitstream")
    version, h, w, bs, nframes, nb = struct.unpack_from("<6I", data, 4)
    if version != VERSION:
        raise ValueError(f"{path}: container version {version}")
    p = 4 + 24
    fts, qps, packed, offs = [], [], [], []
    for _ in range(nframes):
        ft, nqp = struct.unpack_from("<BH", data, p)
        p += 3
        qps.append(np.frombuffer(data, np.int8, nqp, p).astype(int).tolist())
        p += nqp
        (nbytes,) = struct.unpack_from("<I", data, p)
        p += 4
        lens = np.frombuffer(data, np.uint16, nb, p).astype(np.int64)
        p += 2 * nb
        o = np.zeros(nb + 1, np.int64)
        np.cumsum(lens, out=o[1:])
        if o[-1] != nbytes:
            raise ValueError(f"{path}: block lengths do not add up to the frame's byte count")
        fts.append(int(ft))
        offs.append(torch.from_numpy(o.astype(np.int32)).to(device))
        packed.append(torch.frombuffer(bytearray(data[p:p + nbytes]), dtype=torch.uint8).to(device))
        p += nbytes
    if p != len(data):
        raise ValueError(f"{path}: {len(data) - p} bytes after the last frame")
    return {"h": h, "w": w, "bs": bs, "nb": nb, "frame_types": fts, "qp_rows": qps, "packed": packed, "offs": offs}
