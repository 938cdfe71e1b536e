"""Deterministic synthetic Y-plane sequences ("Synthetic input").

The reference reads a CIF 4:2:0 file (main.py:46, video_manager.py:62-77); there is
no network and no dataset here, so every test and benchmark uses this generator.
It is pure numpy (uint64 wrap-around arithmetic), has no RNG-library dependency and
is bit-identical on every host.

Texture:  base(X, Y) = clamp((h(X>>3, Y>>3, seed) & 255)
                             + (h(X, Y, seed ^ 0x9E37) % 17) - 8, 0, 255)
Frame t:  pixel(x, y) = clamp(base(min(x + 2t, W-1), min(y + t, H-1))
                              + (h(x, y, seed ^ (0xA5A5 + t)) % 5) - 2, 0, 255)

i.e. 8x8 random cells plus fixed per-pixel texture noise, moving with a global motion
of (+2, +1) px per frame (inside the +-16 search range), plus +-2 temporal noise so
P-frame residuals are not identically zero.  h() is splitmix64 of the packed
coordinates xor the seed.

Content variants (`content=`, the bench's content-dependence records): the exact SEA search's
speed depends on how well 4x4-cell sums separate candidates, the reference's exhaustive scan
(Encoder.py:688-715) does not.  Only the base texture changes; motion and temporal noise stay:
  "bench"   the texture above (8x8 cells, +-8 pixel noise);
  "lowtex"  32x32 flat cells, +-1 pixel noise: inside a cell every candidate's 4x4 sums agree;
  "noise"   128 + per-pixel noise in [-8, 8], no cells: 4x4 sums of noise barely differ.
"""
from __future__ import annotations

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(z: np.ndarray) -> np.ndarray:
    z = z + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def _h(x: np.ndarray, y: np.ndarray, seed: int) -> np.ndarray:
    key = (y.astype(np.uint64) << np.uint64(32)) | x.astype(np.uint64)
    return _splitmix64(key ^ np.uint64(seed & 0xFFFFFFFFFFFFFFFF))


CONTENTS = ("bench", "lowtex", "noise")
# per content: (cell size log2 or None for no cells, pixel-noise modulus)
_CONTENT = {"bench": (3, 17), "lowtex": (5, 3), "noise": (None, 17)}


def base_texture(height: int, width: int, seed: int, content: str = "bench") -> np.ndarray:
    cl, nm = _CONTENT[content]
    with np.errstate(over="ignore"):
        ys, xs = np.meshgrid(np.arange(height, dtype=np.uint64),
                             np.arange(width, dtype=np.uint64), indexing="ij")
        if cl is None:
            cell = np.full(xs.shape, 128, np.uint64)
        else:
            cell = _h(xs >> np.uint64(cl), ys >> np.uint64(cl), seed) & np.uint64(255)
        noise = _h(xs, ys, seed ^ 0x9E37) % np.uint64(nm)
    v = cell.astype(np.int64) + noise.astype(np.int64) - nm // 2
    return np.clip(v, 0, 255).astype(np.uint8)


def synth_frame(base: np.ndarray, t: int, seed: int) -> np.ndarray:
    height, width = base.shape
    yy = np.minimum(np.arange(height) + t, height - 1)
    xx = np.minimum(np.arange(width) + 2 * t, width - 1)
    moved = base[yy][:, xx].astype(np.int64)
    with np.errstate(over="ignore"):
        ys, xs = np.meshgrid(np.arange(height, dtype=np.uint64),
                             np.arange(width, dtype=np.uint64), indexing="ij")
        tn = _h(xs, ys, seed ^ (0xA5A5 + t)) % np.uint64(5)
    return np.clip(moved + tn.astype(np.int64) - 2, 0, 255).astype(np.uint8)


def synth_sequence(frames: int, height: int, width: int, seed: int = 0, content: str = "bench") -> np.ndarray:
    """uint8 array [frames, height, width] (the reference's y_only_frame_arr, Encoder.py:93)."""
    base = base_texture(height, width, seed, content)
    out = np.empty((frames, height, width), dtype=np.uint8)
    for t in range(frames):
        out[t] = synth_frame(base, t, seed)
    return out


def tie_heavy_sequence(frames: int, height: int, width: int, seed: int = 0) -> np.ndarray:
    """Values in {0, 40, 80, 120} on 4x4 cells: many equal-SAD candidates, which
    exercises the motion-search tie-break (SURVEY.md §8(c) golden vector 2)."""
    with np.errstate(over="ignore"):
        out = np.empty((frames, height, width), dtype=np.uint8)
        ys, xs = np.meshgrid(np.arange(height, dtype=np.uint64),
                             np.arange(width, dtype=np.uint64), indexing="ij")
        for t in range(frames):
            v = _h(xs >> np.uint64(2), ys >> np.uint64(2), seed ^ (t * 7919)) % np.uint64(4)
            out[t] = (v.astype(np.uint8) * 40)
    return out


# ---- the same generator with torch int64 ops (runs on the GPU; bit-identical) ----------
def _s64(c: int) -> int:
    return c - (1 << 64) if c >= (1 << 63) else c


def _t_srl(z, k: int):
    return (z >> k) & ((1 << (64 - k)) - 1)   # logical shift on two's-complement int64


def _t_splitmix64(z):
    z = z + _s64(0x9E3779B97F4A7C15)
    z = (z ^ _t_srl(z, 30)) * _s64(0xBF58476D1CE4E5B9)
    z = (z ^ _t_srl(z, 27)) * _s64(0x94D049BB133111EB)
    return z ^ _t_srl(z, 31)


def _t_umod(z, m: int):
    return ((_t_srl(z, 1) % m) * 2 + (z & 1)) % m


def _t_h(x, y, seed: int):
    return _t_splitmix64(((y << 32) | x) ^ _s64(seed & 0xFFFFFFFFFFFFFFFF))


def synth_sequence_torch(frames: int, height: int, width: int, seed: int = 0, device="cuda",
                         content: str = "bench"):
    """torch.uint8 [frames, height, width] on `device`, equal to synth_sequence()."""
    import torch
    cl, nm = _CONTENT[content]
    ys = torch.arange(height, dtype=torch.int64, device=device)[:, None].expand(height, width)
    xs = torch.arange(width, dtype=torch.int64, device=device)[None, :].expand(height, width)
    cell = torch.full_like(xs, 128) if cl is None else _t_h(xs >> cl, ys >> cl, seed) & 255
    noise = _t_umod(_t_h(xs, ys, seed ^ 0x9E37), nm)
    base = (cell + noise - nm // 2).clamp_(0, 255)
    out = torch.empty((frames, height, width), dtype=torch.uint8, device=device)
    for t in range(frames):
        yy = torch.clamp(torch.arange(height, device=device) + t, max=height - 1)
        xx = torch.clamp(torch.arange(width, device=device) + 2 * t, max=width - 1)
        moved = base[yy][:, xx]
        tn = _t_umod(_t_h(xs, ys, seed ^ (0xA5A5 + t)), 5)
        out[t] = (moved + tn - 2).clamp_(0, 255).to(torch.uint8)
    return out


def write_synth_yuv420(path: str, frames: int, height: int, width: int, seed: int = 0) -> None:
    """A raw planar 4:2:0 file (Y | U | V per frame, the reference's input format,
    video_manager.py:53-77): Y = synth_sequence, U / V = synth_sequence at half size with
    seeds + 1 / + 2."""
    y = synth_sequence(frames, height, width, seed)
    u = synth_sequence(frames, height // 2, width // 2, seed + 1)
    v = synth_sequence(frames, height // 2, width // 2, seed + 2)
    with open(path, "wb") as f:
        for t in range(frames):
            f.write(y[t].tobytes())
            f.write(u[t].tobytes())
            f.write(v[t].tobytes())
