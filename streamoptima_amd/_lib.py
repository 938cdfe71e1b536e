"""ctypes binding of libstreamoptima_hip.so (include/streamoptima.h).

`import torch` happens first so that the library's libamdhip64.so.7 dependency resolves
to the HIP runtime PyTorch already loaded (one runtime per process).  There is no CPU
fallback: if the library is missing or was built for another target, every call raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the CDLL load)

from .build import LIB_PATH

_lock = threading.Lock()
_lib = None

SO_OK = 0
SO_E_INVALID = -1
SO_E_UNSUPPORTED = -2
MAX_REF = 4

_vp = ctypes.c_void_p
_i = ctypes.c_int
_d = ctypes.c_double
_sz = ctypes.c_size_t

_SIGS = {
    "so_abi_version": ([], _i),
    "so_last_error": ([], ctypes.c_char_p),
    "so_me_full_search": ([_vp, _vp, _i, _i, _i, _i, _i, _vp, _vp, _vp], _i),
    "so_inter_tq_recon": ([_vp, _vp, _i, _i, _i, _i, _vp, _vp, _i, _vp, _i, _d, _vp, _vp, _vp, _vp,
                           _vp, _vp, _vp, _vp], _i),
    "so_p_frame_scratch_elems": ([_i, _i, _i, _i], _sz),
    "so_encode_p_frame": ([_vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _i, _d, _vp, _vp, _vp, _vp, _vp,
                           _vp, _vp, _vp, _vp], _i),
    "so_encode_p_rows": ([_vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _i, _d, _vp, _vp, _vp, _vp,
                          _vp, _vp, _vp, _vp, _vp], _i),
    "so_p_run_workspace_elems": ([_i, _i], _sz),
    "so_p_run_resident_workgroups": ([_i], _i),
    "so_p_run_mode_resident_workgroups": ([_i, _i], _i),
    "so_p_run_2pass_fused": ([_i, _i], _i),
    "so_encode_p_run": ([_vp, _i, _vp, _i, _i, _i, _i, _i, _vp, _i, _d, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
                        _i),
    "so_encode_p_run_2pass": ([_vp, _i, _vp, _i, _i, _i, _i, _i, _vp, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                               _vp, _vp, _vp], _i),
    "so_encode_p_runs": ([_vp, _i, _vp, _vp, _i, _i, _i, _i, _i, _vp, _i, _d, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                          _vp], _i),
    "so_i_frame_scratch_elems": ([_i, _i, _i], _sz),
    "so_encode_i_frame": ([_vp, _i, _i, _i, _i, _i, _vp, _i, _d, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                           _vp, _vp], _i),
    "so_encode_i_rows": ([_vp, _i, _i, _i, _i, _i, _i, _i, _vp, _i, _d, _vp, _vp, _vp, _vp, _vp, _vp,
                          _vp, _vp, _vp], _i),
    "so_inter_recon": ([_vp, _i, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp], _i),
    "so_intra_recon": ([_i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp], _i),
    "so_sse_u8": ([_vp, _vp, ctypes.c_int64, _vp, _vp], _i),
    "so_block_xform": ([_vp, _i, _i, _i, _i, _vp, _vp, _vp, _vp], _i),
    "so_encode_p_run_stripe": ([_vp, _i, _vp, _i, _i, _i, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                _i, _vp, _vp, ctypes.c_longlong, _vp, _vp, _vp, _vp, ctypes.c_uint32, _i, _vp], _i),
    "so_stripe_halo_push": ([_vp, _i, _i, _i, _i, _i, _vp, _vp, _vp, _vp, ctypes.c_uint32, _vp], _i),
    "so_alloc_uncached": ([_sz, ctypes.POINTER(ctypes.c_void_p)], _i),
    "so_free_device": ([_vp], _i),
    "so_ipc_export": ([_vp, _vp], _i),
    "so_ipc_open": ([_vp, ctypes.POINTER(ctypes.c_void_p)], _i),
    "so_ipc_close": ([_vp], _i),
    "so_copy_d2d": ([_vp, _vp, _sz, _vp], _i),
    "so_memset_d8": ([_vp, _i, _sz, _vp], _i),
    "so_pack_bound": ([_i, _i], _sz),
    "so_sum_i32_rows": ([_vp, _i, _i, _vp, _vp], _i),
    "so_unpack_frames": ([_i, _vp, _vp, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp], _i),
    "so_encode_p_run_fpipe2": ([_vp, _i, _i, _i, _i, _i, _i, _vp, _i, _d,                 # .. vbs, lam
                                _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,                    # outs, workspace
                                _vp, _vp, _i, _vp, _vp, _vp, _vp, _vp, _i,                 # landing .. nslots
                                ctypes.c_longlong, ctypes.c_uint32, _i, _vp], _i),
    "so_encode_p_run_fpipe_2pass": ([_vp, _i, _i, _i, _i, _i, _i, _vp, _vp, _i, _i,          # .. qp_hi
                                     _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,             # outs, qp maps, ws
                                     _vp, _vp, _i, _vp, _vp, _vp, _vp, _vp, _i,               # landing .. nslots
                                     ctypes.c_longlong, ctypes.c_uint32, _i, _i, _vp], _i),   # .. max_wg p2lag stream
    "so_frame_push": ([_vp, _i, _i, _vp, _vp, ctypes.c_uint32, _vp], _i),
    "so_pack_frames": ([_i, _vp, _vp, _vp, _vp, _i, _i, _vp, _vp, ctypes.c_ulonglong, _vp], _i),
    "so_pack_frames_ex": ([_i, _vp, _vp, _vp, _vp, _i, _i, _vp, _vp, ctypes.c_ulonglong, _vp, _vp], _i),
    "so_fme_plane_stride": ([_i, _i], _sz),
    "so_fme_workspace_bytes": ([_i, _i, _i], _sz),
    "so_fme_planes": ([_vp, _i, _i, _i, _vp, _vp], _i),
    "so_me_search_ex": ([_vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _vp, _vp, _vp], _i),
    "so_encode_p_rows_ex": ([_vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _vp, _i, _d, _i, _i, _i, _vp, _i,
                             _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp], _i),
    "so_inter_recon_ex": ([_vp, _i, _i, _i, _i, _i, _vp, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp], _i),
    "so_encode_i_rows_ex": ([_vp, _i, _i, _i, _i, _i, _i, _i, _vp, _vp, _i, _d, _vp, _vp, _vp, _vp, _vp, _vp,
                             _vp, _vp, _vp], _i),
    "so_intra_recon_ex": ([_i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp], _i),
    "so_qp_map": ([_vp, _i, _i, _i, _i, _i, _i, _vp, _vp, _i, _i, _vp, _vp], _i),
    "so_set_option": ([_i, _i], _i),
    "so_get_option": ([_i], _i),
}

# ME modes (include/streamoptima.h)
ME_FULL, ME_FAST, ME_FAST_PAR = 0, 1, 2
REUSE_ME = 1   # so_encode_p_rows_ex flags
TOKENS_ONLY = 2
# so_set_option (include/streamoptima.h SO_OPT_*)
OPT_RUN_2PASS_FUSED, OPT_FASTME_SERIAL, OPT_FASTME_SEGMENT, OPT_FASTME_WARMUP, OPT_COUNT_SAD_OPS = 1, 2, 3, 4, 5
OPT_RUN_ZERO_SKIP = 7
OPT_TEST_LOSE_FLAG = 6

EXPORTED = tuple(_SIGS)


class HipPathError(RuntimeError):
    """Raised when the gfx950 library is unavailable or a kernel call fails."""


def load(path: str | None = None):
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        p = path or os.environ.get("SO_LIB_PATH") or LIB_PATH   # SO_LIB_PATH: A/B builds (tools/)
        if not os.path.exists(p):
            raise HipPathError(
                f"{p} is missing: build it with `python -m streamoptima_amd.build` (hipcc, gfx950). "
                "There is no CPU fallback for the encode path.")
        lib = ctypes.CDLL(p)
        for name, (args, res) in _SIGS.items():
            if p != LIB_PATH and not hasattr(lib, name):
                continue   # an older A/B build (tools/) without a newer entry point
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = res
        if lib.so_abi_version() != 1:
            raise HipPathError("libstreamoptima_hip.so ABI mismatch")
        _lib = lib
        return lib


def check(rc: int, what: str) -> None:
    if rc != SO_OK:
        msg = load().so_last_error().decode(errors="replace")
        if rc == SO_E_INVALID:
            raise ValueError(f"{what}: {msg}")
        if rc == SO_E_UNSUPPORTED:
            raise NotImplementedError(f"{what}: {msg}")
        raise HipPathError(f"{what}: HIP error {rc}: {msg}")


def set_option(opt: int, value: int) -> int:
    """so_set_option; returns the previous value (raises ValueError on a bad option / value)."""
    lib = load()
    old = lib.so_get_option(opt)
    check(lib.so_set_option(opt, int(value)), "so_set_option")
    return old


class option:
    """Context manager: so_set_option for the duration of a block (tests, A/B tools)."""

    def __init__(self, opt: int, value: int):
        self.opt, self.value, self.old = opt, value, None

    def __enter__(self):
        self.old = set_option(self.opt, self.value)
        return self

    def __exit__(self, *exc):
        set_option(self.opt, self.old)
        return False


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


def ref_array(refs) -> ctypes.Array:
    arr = (ctypes.c_void_p * len(refs))(*[r.data_ptr() for r in refs])
    return arr


def stream_handle(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream
