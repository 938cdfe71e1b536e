"""The C-ABI library: builds for gfx950, loads, exports every declared symbol, and rejects
bad arguments on the host side (no GPU needed for any of this)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "streamoptima.h")).read()
    return sorted(set(re.findall(r"^\s*(?:[\w\*]+\s+)+\*?(so_\w+)\(", src, re.M)))


def test_header_declares_entry_points():
    names = _declared()
    for n in ("so_me_full_search", "so_inter_tq_recon", "so_encode_p_frame", "so_encode_i_frame",
              "so_inter_recon", "so_intra_recon", "so_sse_u8", "so_last_error", "so_abi_version"):
        assert n in names


def test_library_exports_every_declared_symbol():
    from streamoptima_amd import _lib, build
    build.build()
    lib = _lib.load()
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing
    assert set(_lib.EXPORTED) == set(_declared())
    out = subprocess.run(["nm", "-D", "--defined-only", build.LIB_PATH], capture_output=True, text=True).stdout
    for n in _declared():
        assert re.search(rf"\bT {n}\b", out), n


def test_ctypes_signatures_match_the_header():
    """Every ctypes signature in _lib._SIGS has the header declaration's parameter count and
    pointer / integer / floating kinds (a shifted argument would pass a size as a pointer)."""
    from streamoptima_amd import _lib
    hdr = open(os.path.join(ROOT, "include", "streamoptima.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    ptr_types = (ctypes.c_void_p, ctypes.c_char_p) + tuple(t for t in vars(ctypes).values()
                                                         if isinstance(t, type) and t.__name__.startswith("LP_"))
    for name, (args, _) in _lib._SIGS.items():
        m = re.search(r"^\s*(?:int|size_t|const char\*)\s+" + name + r"\(([^;]*?)\);", hdr, re.M | re.S)
        assert m, name
        params = [p.strip() for p in m.group(1).split(",") if p.strip() and p.strip() != "void"]
        assert len(params) == len(args), (name, len(params), len(args))
        for i, (p, a) in enumerate(zip(params, args)):
            is_ptr = "*" in p
            if is_ptr:
                assert a in ptr_types or issubclass(a, ctypes._Pointer), (name, i, p, a)
            elif "double" in p:
                assert a is ctypes.c_double, (name, i, p, a)
            else:
                assert a in (ctypes.c_int, ctypes.c_uint32, ctypes.c_int64, ctypes.c_longlong, ctypes.c_size_t,
                             ctypes.c_ulonglong, ctypes.c_int32), (name, i, p, a)


def test_code_object_is_gfx950():
    from streamoptima_amd import build
    blob = open(build.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_host_side_validation_without_gpu():
    from streamoptima_amd import _lib
    lib = _lib.load()
    bad = lib.so_encode_p_frame(None, None, 1, 64, 64, 12, 16, 4, None, 0, 0.0, None, None, None, None, None,
                                None, None, None, None)
    assert bad == _lib.SO_E_UNSUPPORTED
    assert b"block_size 12" in lib.so_last_error()
    bad = lib.so_encode_i_frame(None, 60, 64, 16, 16, 4, None, 0, 0.0, None, None, None, None, None, None, None,
                                None, None)
    assert bad == _lib.SO_E_INVALID
    assert lib.so_p_frame_scratch_elems(2160, 3840, 16, 1) == 32400 * 20 + 2 * 4096 * 6   # + fast-ME segments
    assert lib.so_i_frame_scratch_elems(64, 64, 16) == 16 * 256 + 16 * 8
    with pytest.raises(NotImplementedError):
        _lib.check(lib.so_me_full_search(None, None, 1, 64, 64, 16, 99, None, None, None), "me")


def test_p_runs_validation_without_gpu():
    """so_encode_p_runs refuses a frame whose in-list reference is not an earlier frame (the
    persistent launch takes frames in list order: a later reference could deadlock it) and an
    output plane that aliases a reference -- before anything touches the GPU."""
    import ctypes
    from streamoptima_amd import _lib
    lib = _lib.load()
    n = 2
    fake = [ctypes.c_void_p(0x1000 * (i + 1)) for i in range(12)]

    def arr(*ps):
        return (ctypes.c_void_p * n)(*ps)
    cur = arr(fake[0], fake[1])
    outs = [arr(fake[2 + 2 * k], fake[3 + 2 * k]) for k in range(5)]

    def call(refs, ref_frame, recon, vbs=0, lam=0.0):
        return lib.so_encode_p_runs(cur, n, refs, (ctypes.c_int32 * n)(*ref_frame), 64, 128, 16, 16, 4, None, vbs,
                                    lam, outs[0], outs[1], outs[2], outs[3], outs[4], recon, None,
                                    ctypes.c_void_p(0x9000), None)
    recon = arr(fake[10], fake[11])
    assert call(arr(fake[8], fake[9]), [-1, 1], recon) == _lib.SO_E_INVALID
    assert b"ref_frame[1]" in lib.so_last_error()
    assert call(arr(fake[8], None), [-1, -1], recon) == _lib.SO_E_INVALID
    assert call(arr(fake[10], None), [-1, 0], recon) == _lib.SO_E_INVALID
    assert b"aliases" in lib.so_last_error()
    assert call(arr(fake[8], None), [-1, 0], recon, vbs=2) == _lib.SO_E_INVALID
    assert call(arr(fake[8], None), [-1, 0], recon, vbs=1, lam=float("nan")) == _lib.SO_E_INVALID
    assert b"lambda" in lib.so_last_error()
    assert lib.so_encode_p_runs(cur, n, arr(fake[8], None), (ctypes.c_int32 * n)(-1, 0), 64, 96, 16, 16, 4, None, 0,
                                0.0, outs[0], outs[1], outs[2], outs[3], outs[4], recon, None, ctypes.c_void_p(0x9000),
                                None) == _lib.SO_E_UNSUPPORTED


def test_two_pass_run_and_frame_pipe_validation_without_gpu():
    """so_encode_p_run_2pass and so_encode_p_run_fpipe2 reject unsupported geometry, a bad QP
    clamp, a reconstruction aliasing the reference or lying in the landing planes, a short
    landing stride, a push code below -1 or past the peers' slots and a run past the landing
    slots -- on the host, before any launch."""
    from streamoptima_amd import _lib
    lib = _lib.load()
    n, H, W = 2, 64, 128
    fake = [ctypes.c_void_p(0x100000 * (i + 1)) for i in range(16)]

    def arr(*ps):
        return (ctypes.c_void_p * n)(*ps)
    cur = arr(fake[0], fake[1])
    outs = [arr(fake[2 + 2 * k], fake[3 + 2 * k]) for k in range(5)]
    qmap = arr(fake[12], fake[13])
    ws = ctypes.c_void_p(0x9000)

    def two_pass(ref0, recon, bs=16, w=W, lo=0, hi=20):
        return lib.so_encode_p_run_2pass(cur, n, ref0, H, w, bs, 16, 4, None, None, lo, hi, outs[0], outs[1], outs[2],
                                         outs[3], outs[4], recon, None, qmap, ws, None)
    recon = arr(fake[10], fake[11])
    assert two_pass(fake[14], recon, bs=8) == _lib.SO_E_UNSUPPORTED
    assert two_pass(fake[14], recon, w=96) == _lib.SO_E_UNSUPPORTED
    assert two_pass(fake[14], recon, lo=5, hi=3) == _lib.SO_E_INVALID
    assert b"QP clamp" in lib.so_last_error()
    assert two_pass(fake[10], recon) == _lib.SO_E_INVALID
    assert b"aliases" in lib.so_last_error()

    stride = H * W
    land0, land_flags = 0x4000000, ctypes.c_void_p(0x5000000)

    def fpipe(recon, push, stride=stride, slot0=0, nslots=3):
        return lib.so_encode_p_run_fpipe2(cur, n, H, W, 16, 16, 4, None, 0, 0.0, outs[0], outs[1], outs[2], outs[3],
                                          outs[4],
                                          recon, None, ws, ctypes.c_void_p(land0), land_flags, slot0, fake[14],
                                          fake[15], fake[14], fake[15], (ctypes.c_int32 * n)(*push), nslots, stride,
                                          1, 0, None)
    assert fpipe(recon, [0, 2], stride=stride - 1) == _lib.SO_E_INVALID
    assert fpipe(recon, [0, 2], slot0=-1) == _lib.SO_E_INVALID
    assert fpipe(recon, [0, -2]) == _lib.SO_E_INVALID
    assert b"push_to[1]" in lib.so_last_error()
    assert fpipe(recon, [0, 6]) == _lib.SO_E_INVALID            # slot 3 of a peer with 3 slots
    assert b"push_to[1]" in lib.so_last_error()
    assert fpipe(recon, [0, 2], slot0=2) == _lib.SO_E_INVALID   # slots 2, 3 of 3
    assert b"nslots" in lib.so_last_error()
    assert fpipe(arr(fake[10], ctypes.c_void_p(land0 + stride)), [0, 2]) == _lib.SO_E_INVALID
    assert b"landing planes" in lib.so_last_error()

    def fpipe2p(push, p2lag=0, lo=0, hi=12):
        return lib.so_encode_p_run_fpipe_2pass(cur, n, H, W, 16, 16, 4, None, None, lo, hi, outs[0], outs[1], outs[2],
                                               outs[3], outs[4], recon, None, qmap, ws, ctypes.c_void_p(land0),
                                               land_flags, 0, fake[14], fake[15], fake[14], fake[15],
                                               (ctypes.c_int32 * n)(*push), 3, stride, 1, 0, p2lag, None)
    assert fpipe2p([0, 2], p2lag=-1) == _lib.SO_E_INVALID
    assert b"p2lag" in lib.so_last_error()
    assert fpipe2p([0, 2], lo=7, hi=3) == _lib.SO_E_INVALID
    assert fpipe2p([0, 8]) == _lib.SO_E_INVALID
    assert b"push_to[1]" in lib.so_last_error()


def test_product_never_imports_the_oracle():
    pkg = os.path.join(ROOT, "streamoptima_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                text = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in re.sub(r"#.*|//.*", "", text).replace("oracles", ""), f
