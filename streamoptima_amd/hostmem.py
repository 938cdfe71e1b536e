"""Page-locked host buffers for the PCIe legs (BASELINE.md section 4's region).

torch's pinned allocator (hipHostMalloc) gave the GPU box's 4K GOP upload 49-57 GB/s from one
allocation to the next (the copy engine's rate from the same kind of buffer varied with where
and when it was allocated: tools/s4_probe.py, s4_probe2.py, profiles/r06/s4_probe*.log), while
anonymous memory mapped and first touched by this process, then registered with
hipHostRegister, read at 57.5 GB/s.  pinned_empty() returns such a buffer as a CPU tensor
(is_pinned() is True).  The mapping stays registered for the life of the process.
device_ptr() is the address a kernel stores to such a buffer through (so_pack_frames_ex's
totals).
"""
from __future__ import annotations

import ctypes
import mmap
import os
import threading

import numpy as np
import torch

_LOCK = threading.Lock()
_KEEP: list = []      # (mmap, address, size): alive and registered until the process ends
_HUGE = 2 << 20


def _hip():
    return ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))


def pinned_empty(shape, dtype=torch.uint8) -> torch.Tensor:
    """A page-locked host tensor of `shape` / `dtype` (uninitialised contents are zeros)."""
    n = int(np.prod(shape)) * torch.empty((), dtype=dtype).element_size()
    size = max(_HUGE, -(-n // _HUGE) * _HUGE)
    m = mmap.mmap(-1, size + _HUGE)
    if hasattr(mmap, "MADV_HUGEPAGE"):
        m.madvise(mmap.MADV_HUGEPAGE)
    base = ctypes.addressof(ctypes.c_char.from_buffer(m))
    off = (-base) % _HUGE
    flat = np.frombuffer(m, dtype=np.uint8, count=size, offset=off)
    flat[::4096] = 0                       # first touch by this process: pages placed now
    rc = _hip().hipHostRegister(ctypes.c_void_p(base + off), ctypes.c_size_t(size), ctypes.c_uint(0))
    if rc != 0:
        raise RuntimeError(f"hipHostRegister failed ({rc}) for a {size}-byte host buffer")
    with _LOCK:
        _KEEP.append((m, base + off, size))
    t = torch.from_numpy(flat[:n]).view(dtype)
    return t.view(shape) if len(tuple(shape)) else t


def device_ptr(t: torch.Tensor) -> int:
    """The device address of page-locked host tensor t's first element (hipHostGetDevicePointer)."""
    if t.device.type != "cpu" or not t.is_pinned():
        raise ValueError("device_ptr: a page-locked host tensor is required")
    p = ctypes.c_void_p()
    rc = _hip().hipHostGetDevicePointer(ctypes.byref(p), ctypes.c_void_p(t.data_ptr()), ctypes.c_uint(0))
    if rc != 0 or not p.value:
        raise RuntimeError(f"hipHostGetDevicePointer failed ({rc})")
    return int(p.value)
