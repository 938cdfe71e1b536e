"""Streams on hardware queues of their own.

HIP maps a process's streams onto at most GPU_MAX_HW_QUEUES (4 on the GPU boxes) hardware
queues, round-robin in creation order, and torch.cuda.Stream() hands out streams from a pool
of its own.  Two streams that land on one queue are serialised by it: a stream's wait on
another stream's event parks the whole queue, including the other stream's work behind it.
Which streams collide therefore depends on how many streams the process created before --
the reason BASELINE.md section 4's region (three engines overlapped: H2D copies, kernels,
D2H copies) read 5.7 ms per 4K GOP when measured first in bench.py and 9.5 ms (= upload +
encode + download, back to back) after the records had created their streams.

A stream created with a CU mask gets a hardware queue of its own
(hipExtStreamCreateWithCUMask; the mask here is every CU, so it restricts nothing).  The
streams are created once per (device, role) and kept for the life of the process.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

_LOCK = threading.Lock()
_STREAMS: dict = {}
_HIP = None


def _hip():
    global _HIP
    if _HIP is None:
        # the HIP runtime torch itself loaded (one runtime per process)
        _HIP = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    return _HIP


def dedicated_stream(device, role: str) -> torch.cuda.ExternalStream:
    """The process's stream for `role` on `device`, on a hardware queue no other stream
    shares (created on first use)."""
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    key = (idx, role)
    with _LOCK:
        s = _STREAMS.get(key)
        if s is None:
            hip = _hip()
            ncu = torch.cuda.get_device_properties(idx).multi_processor_count
            words = (ncu + 31) // 32
            mask = (ctypes.c_uint32 * words)(*([0xFFFFFFFF] * words))
            h = ctypes.c_void_p()
            with torch.cuda.device(idx):
                rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(words), mask)
            if rc != 0:
                raise RuntimeError(f"hipExtStreamCreateWithCUMask failed ({rc}) for the {role!r} stream")
            s = _STREAMS[key] = torch.cuda.ExternalStream(h.value, device=torch.device("cuda", idx))
        return s
