"""GPU parity: the gfx950 path (through the C-ABI) against the reference's golden vectors
and against the C oracle.  Bar: bit-exact for every integer output (MVs, split flags,
QTC, token counts, reconstructions); PSNR from the same integer SSE."""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, golden

pytestmark = pytest.mark.gpu


def _dev(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _plane(a, dev):
    from streamoptima_amd.engine import alloc_planes
    a = np.ascontiguousarray(a, dtype=np.uint8)
    p = alloc_planes(1, *a.shape, dev)[0]
    p.copy_(torch.from_numpy(a))
    return p


def _me(cur, refs, bs, sr, dev, sub=False):
    from streamoptima_amd import _lib
    lib = _lib.load()
    h, w = cur.shape
    nb = (h // bs) * (w // bs)
    c = _plane(cur, dev)
    rs = [_plane(r, dev) for r in refs]
    best = torch.empty((nb, 4), dtype=torch.int32, device=dev)
    subt = torch.empty((nb, 4, 4), dtype=torch.int32, device=dev) if sub else None
    rc = lib.so_me_full_search(c.data_ptr(), _lib.ref_array(rs), len(rs), h, w, bs, sr, best.data_ptr(),
                               _lib.ptr(subt), _lib.stream_handle())
    _lib.check(rc, "so_me_full_search")
    torch.cuda.synchronize()
    return best.cpu().numpy(), (subt.cpu().numpy() if sub else None)


def _sym_host(sym):
    from streamoptima_amd.package import symbols_to_host
    return symbols_to_host(sym)


def _assert_frame(host, ref, keys=("split", "mv", "qtc", "tokens", "recon")):
    for k in keys:
        a, b = host[k], ref[k]
        if k == "recon":
            a = a[: b.shape[0], : b.shape[1]]
        assert a.shape == b.shape, (k, a.shape, b.shape)
        bad = np.argwhere(a != b)
        assert bad.size == 0, f"{k}: {len(bad)} mismatches, first at {bad[:3].tolist()}"


# ---------------------------------------------------------------- golden vectors (reference)
def test_me_tie_golden_16(gpu):
    g = golden("me_tie.npz")
    best, _ = _me(g["cur"], [g["ref"]], 16, 16, gpu)
    exp = g["best16"].reshape(-1, 4)
    assert (best == exp).all(), np.argwhere(best != exp)[:5]


def test_me_tie_golden_8x8_two_refs(gpu):
    g = golden("me_tie.npz")
    best, _ = _me(g["cur"], [g["ref"], g["ref2"]], 8, 16, gpu)
    exp = g["best8"]                       # 12 rows x 44 cols of 8x8 blocks
    got = best.reshape(36, 44, 4)[:12]
    assert (got == exp).all(), np.argwhere(got != exp)[:5]


@pytest.mark.parametrize("name,vbs,rc", [("cif_p_vbs0.npz", False, False), ("cif_p_vbs1.npz", True, False),
                                         ("cif_p_vbs1_rc.npz", True, True)])
def test_inter_frame_golden(gpu, name, vbs, rc):
    from streamoptima_amd.engine import Engine
    g = golden(name)
    eng = Engine(288, 352, 16, 16, vbs, 0.015, gpu)
    qp_row = g["qp_per_row"].tolist() if rc else None
    sym = eng.encode_p(_plane(g["cur"], gpu), [_plane(g["ref"], gpu)], 4, qp_row)
    torch.cuda.synchronize()
    h = _sym_host(sym)
    _assert_frame(h, {k: g[k] for k in ("split", "mv", "qtc", "tokens", "recon")})
    avg = (int(h["mae_num"].sum()) / 256) / len(h["mae_num"])
    assert avg == float(g["avg_mae"])
    assert int(h["tokens"].sum()) == int(g["residual_size"])


@pytest.mark.parametrize("name,vbs,qp,hw", [("cif_i_qp6_vbs0.npz", False, 6, (288, 352)),
                                            ("cif_i_qp6_vbs1.npz", True, 6, (288, 352)),
                                            ("i_64x128_vbs1.npz", True, 3, (64, 128))])
def test_intra_frame_golden(gpu, name, vbs, qp, hw):
    from streamoptima_amd.engine import Engine
    g = golden(name)
    eng = Engine(hw[0], hw[1], 16, 16, vbs, 0.015, gpu)
    sym = eng.encode_i(_plane(g["cur"], gpu), qp)
    torch.cuda.synchronize()
    h = _sym_host(sym)
    _assert_frame(h, {k: g[k] for k in ("split", "mv", "qtc", "tokens", "recon")})
    assert (int(h["mae_num"].sum()) / 256) / len(h["mae_num"]) == float(g["avg_mae"])


GOPS = [
    ("gop_cif_vbs0", dict(qp=4, intra_dur=4, vbs=False)),
    ("gop_cif_vbs1_rc1", dict(qp=4, intra_dur=3, vbs=True, rc=1, target="2 mbps")),
    ("gop_small_rc2", dict(qp=3, intra_dur=4, vbs=True, rc=2, target="1 mbps", intra_thresh=150)),
]


@pytest.mark.parametrize("name,cfg", GOPS)
def test_gop_golden(gpu, name, cfg, tmp_path, monkeypatch):
    from streamoptima_amd.Encoder import Y_Video_codec
    g = golden(name + ".npz")
    frames = g["frames"]
    f, h, w = frames.shape
    tables = json.load(open(os.path.join(GOLDEN, "rc_schedule.json")))["tables"]
    monkeypatch.chdir(tmp_path)
    enc = Y_Video_codec(h, w, f, 16, 16, cfg["qp"], cfg["intra_dur"], 0, 0.015, cfg["vbs"], nRefFrames=1,
                        y_only_frame_arr=frames, RCFlag=cfg.get("rc"), targetBR=cfg.get("target"),
                        qp_rate_tables=tables, intra_thresh=cfg.get("intra_thresh"), device=gpu)
    psnr = enc.encode(block_size=16)
    assert np.allclose(psnr, g["psnr"], rtol=0, atol=1e-9), (psnr, g["psnr"])
    pkg = enc.encoded_package
    assert pkg["frame_type_seq"] == g["frame_type"].tolist()
    for i in range(f):
        assert pkg["Qp_per_row_per_frame"][i] == g[f"qp_per_row{i}"].tolist()
        hsym = _sym_host(enc._symbols[i])
        _assert_frame(hsym, {"split": g[f"split{i}"], "mv": g[f"mv{i}"], "qtc": g[f"qtc{i}"],
                             "tokens": g[f"tokens{i}"], "recon": g["recon"][i]})
        dec = enc.decoded_device[i].cpu().numpy()
        assert (dec == g["decoded"][i]).all()
    # text bitstream of the package == the reference's lines
    import gzip
    js = json.load(gzip.open(os.path.join(GOLDEN, name + "_bitstream.json.gz"), "rt"))
    for i in range(f):
        ft = pkg["frame_type_seq"][i]
        line = f"{ft}|" + enc.differential_encoder_frame(ft, pkg["MVS per Frame"][i], pkg["Qp_per_row_per_frame"][i])
        assert line == js["mv_lines"][i]
        assert enc.entropy_encoder_frame(pkg["approx residual"][i], 16) == js["residual_lines"][i]


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("key,h,w", [("1920x1088", 1088, 1920), ("3840x2160", 2160, 3840)])
def test_large_hashes(gpu, key, h, w, tmp_path, monkeypatch):
    """2-frame I+P encodes at 1088p and 4K against the reference's sha256 (QTC, MV, split,
    recon) — the reference needed ~340 s for the 4K pair."""
    from streamoptima_amd.Encoder import Y_Video_codec
    from streamoptima_amd.synth import synth_sequence
    exp = json.load(open(os.path.join(GOLDEN, "large_hashes.json")))[key]
    seq = synth_sequence(2, h, w, seed=0)
    monkeypatch.chdir(tmp_path)
    enc = Y_Video_codec(h, w, 2, 16, 16, 4, 2, 0, 0.015, False, y_only_frame_arr=seq, device=gpu)
    psnr = enc.encode(block_size=16)
    assert np.allclose(psnr, exp["psnr"], rtol=0, atol=1e-9)
    for i in range(2):
        hs = _sym_host(enc._symbols[i])
        assert _sha(hs["split"]) == exp[f"split{i}"]
        assert _sha(hs["mv"]) == exp[f"mv{i}"]
        assert _sha(hs["qtc"]) == exp[f"qtc{i}"]
        assert int(hs["tokens"].sum()) == exp[f"tokens{i}"]
        assert _sha(hs["recon"]) == exp[f"recon{i}"]


# ---------------------------------------------------------------- GPU vs C oracle
def _frames(kind, h, w, seed, n=2):
    from streamoptima_amd.synth import synth_sequence, tie_heavy_sequence
    return tie_heavy_sequence(n, h, w, seed) if kind == "tie" else synth_sequence(n, h, w, seed)


CASES = [
    # (h, w, bs, sr, vbs, nref, qp, kind)
    (64, 64, 16, 16, False, 1, 4, "synth"),
    (64, 64, 16, 16, True, 1, 0, "synth"),
    (48, 80, 16, 16, True, 2, 2, "tie"),
    (128, 96, 16, 16, True, 3, 5, "synth"),
    (32, 32, 16, 16, False, 1, 4, "synth"),
    (16, 16, 16, 16, False, 1, 4, "synth"),       # no valid candidate: boundary path
    (64, 48, 8, 16, False, 1, 3, "synth"),
    (40, 56, 8, 16, False, 2, 1, "tie"),
    (64, 64, 16, 7, False, 1, 4, "synth"),        # generic ME path (sr != 16)
    (64, 80, 16, 5, True, 2, 3, "tie"),
    (256, 272, 16, 16, True, 1, 4, "synth"),      # more than one ME tile
    (64, 64, 8, 8, False, 1, 3, "synth"),         # 8x8 blocks, sr <= bs: the intra scan at BS 8
    (48, 40, 8, 8, False, 1, 2, "tie"),           # W % 16 != 0: the sequential intra walk
    (32, 1024, 8, 8, False, 1, 4, "synth"),       # 128 blocks a row: 32 chunks of 4 (intra scan)
    (32, 2048, 16, 16, False, 1, 4, "tie"),       # 128 blocks a row: 16 chunks of 8 over 4 waves
]


@pytest.mark.parametrize("h,w,bs,sr,vbs,nref,qp,kind", CASES)
def test_inter_vs_oracle(gpu, h, w, bs, sr, vbs, nref, qp, kind):
    from oracle import oracle as O
    from streamoptima_amd.engine import Engine
    seq = _frames(kind, h, w, 11 + h + w, n=nref + 1)
    cur, refs = seq[nref], [seq[k] for k in range(nref)]
    rng = np.random.default_rng(h * w)
    qp_row = rng.integers(0, 7, size=h // bs).tolist()
    for qr in (None, qp_row):
        exp = O.inter_frame(cur, refs, bs, sr, qp, qr, vbs, 0.015)
        eng = Engine(h, w, bs, sr, vbs, 0.015, gpu)
        sym = eng.encode_p(_plane(cur, gpu), [_plane(r, gpu) for r in refs], qp, qr)
        torch.cuda.synchronize()
        hs = _sym_host(sym)
        _assert_frame(hs, exp)
        assert (hs["mae_num"] == exp["mae_num"]).all()


@pytest.mark.parametrize("h,w,bs,sr,vbs,nref,qp,kind", CASES)
def test_intra_vs_oracle(gpu, h, w, bs, sr, vbs, nref, qp, kind):
    from oracle import oracle as O
    from streamoptima_amd.engine import Engine
    cur = _frames(kind, h, w, 5 + h, n=1)[0]
    rng = np.random.default_rng(h + w)
    qp_row = rng.integers(0, 7, size=h // bs).tolist()
    for qr in (None, qp_row):
        exp = O.intra_frame(cur, bs, sr, qp, qr, vbs, 0.015)
        eng = Engine(h, w, bs, sr, vbs, 0.015, gpu)
        sym = eng.encode_i(_plane(cur, gpu), qp, qr)
        torch.cuda.synchronize()
        hs = _sym_host(sym)
        _assert_frame(hs, exp)
        assert (hs["mae_num"] == exp["mae_num"]).all()


def test_decoder_matches_encoder_recon(gpu, tmp_path, monkeypatch):
    """decoder.decode over the package lists == the encoder's reconstruction (closed loop).
    nRefFrames=1: with more references the reference's own decoder disagrees with its
    encoder (it clears the list on I-frames, decoder.py:520 vs Encoder.py:1864)."""
    from streamoptima_amd.Encoder import Y_Video_codec
    from streamoptima_amd.synth import synth_sequence
    seq = synth_sequence(5, 96, 160, seed=4)
    monkeypatch.chdir(tmp_path)
    enc = Y_Video_codec(96, 160, 5, 16, 16, 3, 3, 0, 0.015, True, nRefFrames=1, y_only_frame_arr=seq, device=gpu)
    enc.encode(block_size=16)
    pkg = enc.encoded_package
    dec = enc.decoder.decode(pkg["frame_type_seq"], pkg["approx residual"], pkg["Qp_per_row_per_frame"],
                             pkg["MVS per Frame"], 0, 3, 16, 5, 160, 96)
    for i in range(5):
        assert (dec[i] == enc._symbols[i].recon.cpu().numpy()).all()
        assert torch.equal(enc.decoded_device[i], enc._symbols[i].recon)


def test_gop_vs_oracle_multiref(gpu, tmp_path, monkeypatch):
    from oracle.gop import encode_gop
    from streamoptima_amd.Encoder import Y_Video_codec
    from streamoptima_amd.synth import synth_sequence
    seq = synth_sequence(6, 80, 112, seed=9)
    exp = encode_gop(seq, 2, 4, vbs=True, nref=3)
    monkeypatch.chdir(tmp_path)
    enc = Y_Video_codec(80, 112, 6, 16, 16, 2, 4, 0, 0.015, True, nRefFrames=3, y_only_frame_arr=seq, device=gpu)
    psnr = enc.encode(block_size=16)
    for i in range(6):
        hs = _sym_host(enc._symbols[i])
        assert hs["frame_type"] == exp[i]["frame_type"]
        _assert_frame(hs, exp[i])
        assert psnr[i] == exp[i]["psnr"]


def test_full_size_properties_4k(gpu):
    """4K P-frame at full size: decoder(encoder symbols) == encoder recon, residual_size ==
    sum(tokens), every MV inside the search range and the strict bound."""
    from streamoptima_amd.engine import Engine
    from streamoptima_amd.synth import synth_sequence
    h, w = 2160, 3840
    seq = synth_sequence(2, h, w, seed=1)
    eng = Engine(h, w, 16, 16, True, 0.015, gpu)
    ref = _plane(seq[0], gpu)
    sym = eng.encode_p(_plane(seq[1], gpu), [ref], 4)
    rec = eng.recon_inter([ref], sym.split, sym.mv, sym.qtc, 4)
    torch.cuda.synchronize()
    assert torch.equal(rec, sym.recon)
    mv = sym.mv.cpu().numpy()
    assert np.abs(mv[..., :2]).max() <= 16
    nbx = w // 16
    bx = np.arange(mv.shape[0]) % nbx * 16
    unsplit = sym.split.cpu().numpy() == 0
    assert ((bx + mv[:, 0, 0])[unsplit] < w - 16).all()


# ---------------------------------------------------------------- stripes (multi-GPU sharding)
@pytest.mark.parametrize("h,w,vbs,frame_type", [(256, 272, True, 1), (256, 272, False, 0), (208, 160, True, 0),
                                                (2160, 3840, False, 1)])
def test_stripes_concatenate_to_full_frame(gpu, h, w, vbs, frame_type):
    """so_encode_p_rows / so_encode_i_rows over every rank's [by0, by1) for world sizes
    2, 3 and 8: the rank-order concatenation equals so_encode_*_frame bit for bit, and
    the stripe reconstructions tile the full one."""
    from streamoptima_amd.dist import stripe_rows
    from streamoptima_amd.engine import Engine, alloc_planes
    from streamoptima_amd.synth import synth_sequence
    seq = synth_sequence(2, h, w, seed=h + w)
    eng = Engine(h, w, 16, 16, vbs, 0.015, gpu)
    cur, ref = _plane(seq[1], gpu), _plane(seq[0], gpu)
    qr = np.random.default_rng(w).integers(0, 7, size=h // 16).tolist()
    qdev = eng.qp_row_tensor(qr)
    full = eng.encode_p(cur, [ref], 3, qr) if frame_type else eng.encode_i(cur, 3, qr)
    torch.cuda.synchronize()
    for world in (2, 3, 8):
        plane = alloc_planes(1, h, w, gpu, fill=0)[0]
        parts = []
        for rank in range(world):
            by0, by1, _ = stripe_rows(eng.nby, world, rank)
            if by1 == by0:
                continue
            s = eng.new_stripe_symbols(frame_type, by0, by1, plane)
            if frame_type:
                eng.encode_p_rows(cur, [ref], by0, by1, 3, s, qp_row_dev=qdev)
            else:
                eng.encode_i_rows(cur, by0, by1, 3, s, qp_row_dev=qdev)
            parts.append(s)
        torch.cuda.synchronize()
        for k in ("split", "mv", "qtc", "tokens", "mae_num"):
            cat = torch.cat([getattr(p, k) for p in parts])
            assert torch.equal(cat, getattr(full, k)), (world, k)
        assert torch.equal(plane, full.recon), world
        assert sum(int(p.sse.sum()) for p in parts) == int(full.sse.sum())


def test_stripe_gop_encoder_single_rank(gpu):
    """StripeGOPEncoder with one rank (no process group) == Y_Video_codec.encode_device."""
    from streamoptima_amd.Encoder import Y_Video_codec
    from streamoptima_amd.dist import StripeGOPEncoder
    from streamoptima_amd.engine import alloc_planes
    from streamoptima_amd.synth import synth_sequence_torch
    h, w, f = 128, 192, 4
    codec = Y_Video_codec(h, w, f, 16, 16, 4, 3, 0, 0.015, True, y_only_frame_arr=None, device=gpu)
    frames = alloc_planes(f, h, w, gpu)
    frames.copy_(synth_sequence_torch(f, h, w, seed=2, device=gpu))
    a = codec.encode_device(frames, 3)
    b = StripeGOPEncoder(codec.engine()).encode(frames, 3, 4)
    torch.cuda.synchronize()
    assert torch.equal(a["sse"], b["sse"])
    for sa, sb in zip(a["symbols"], b["symbols"]):
        assert sa.frame_type == sb.frame_type
        for k in ("split", "mv", "qtc", "tokens", "mae_num", "recon"):
            assert torch.equal(getattr(sa, k), getattr(sb, k)), k


# ---------------------------------------------------------------- ME search paths (SEA / dense fallback)
@pytest.mark.parametrize("kind", ["flat", "noise", "synth", "tie", "ramp"])
def test_me_paths_vs_oracle(gpu, kind):
    """The default bs-16 ME prunes candidates by 4x4-sum lower bounds (me_sea2_kernel) and falls
    back to every candidate's SAD when too many survive.  Flat frames make every candidate survive
    (fallback), noise gives weak bounds, tie-heavy and ramp content stress the tie-break.
    Every block's (dx, dy, ref, SAD) must equal the oracle's exhaustive search."""
    from oracle import oracle as O
    from streamoptima_amd.synth import synth_sequence, tie_heavy_sequence
    h, w = 96, 160
    rng = np.random.default_rng(7)
    if kind == "flat":
        seq = np.full((2, h, w), 77, np.uint8)
    elif kind == "noise":
        seq = rng.integers(0, 256, size=(2, h, w), dtype=np.uint8)
    elif kind == "ramp":
        yy, xx = np.mgrid[0:h, 0:w]
        base = ((xx * 3 + yy * 5) % 256).astype(np.uint8)
        seq = np.stack([base, np.roll(base, (2, -3), axis=(0, 1))])
    elif kind == "tie":
        seq = tie_heavy_sequence(2, h, w, 3)
    else:
        seq = synth_sequence(2, h, w, 5)
    best, _ = _me(seq[1], [seq[0]], 16, 16, gpu)
    nbx = w // 16
    for b in range(best.shape[0]):
        x, y = (b % nbx) * 16, (b // nbx) * 16
        exp = O.me_block(seq[1], [seq[0]], x, y, 16, 16)
        assert tuple(int(v) for v in best[b]) == exp, (kind, b, tuple(best[b]), exp)


# ---------------------------------------------------------------- FME and fast ME
# reference goldens (tests/golden/make_golden.py --only fme,gopme) and the C oracle
ME_VARIANTS = ["fme_cif_vbs0", "fme_96x128_vbs1", "fme_64x96_sr4_vbs1", "fme_64x96_nref2", "fast_cif_vbs0",
               "fast_cif_vbs1", "fast_cif_nref2_vbs1", "fast_fme_cif_vbs1", "fast_par2_cif"]


def _me_mode(fast, pm):
    return 0 if not fast else (2 if pm == 2 else 1)


@pytest.mark.parametrize("name", ME_VARIANTS)
def test_inter_me_variants_golden(gpu, name):
    """complete_inter_flow with FMEEnable / fast_me (and fast_me under ParallelMode 2)."""
    from streamoptima_amd.engine import Engine
    g = golden("inter_me_variants.npz")
    h, w, sr, vbs, fast, fme, nref, pm = (int(v) for v in g[f"{name}__cfg"])
    eng = Engine(h, w, 16, sr, bool(vbs), 0.015, gpu, me_mode=_me_mode(fast, pm), fme=bool(fme))
    refs = [_plane(r, gpu) for r in g[f"{name}__refs"]]
    sym = eng.encode_p(_plane(g[f"{name}__cur"], gpu), refs, 4)
    torch.cuda.synchronize()
    hs = _sym_host(sym)
    _assert_frame(hs, {k: g[f"{name}__{k}"] for k in ("split", "mv", "qtc", "tokens", "recon")})
    m = hs["mae_num"]
    avg = float("inf") if (m < 0).any() else (int(m.sum()) / 256) / len(m)
    assert avg == float(g[f"{name}__avg_mae"])
    if fme:   # the decoder's FME recon of the same symbols
        rec = eng.recon_inter(refs, sym.split, sym.mv, sym.qtc, 4)
        torch.cuda.synchronize()
        assert (rec.cpu().numpy() == g[f"{name}__recon"]).all()


def test_fme_planes_golden(gpu):
    """so_fme_planes == frac_me_reference_frame, interleaved back (wrap and no-wrap)."""
    from streamoptima_amd import _lib
    lib = _lib.load()
    g = golden("fme_frames.npz")
    h, w = g["a"].shape
    ps = lib.so_fme_plane_stride(h, w)
    for src, wrap, key in ((g["a"], 1, "up_u8_a"), (g["b"], 1, "up_u8_b"), (g["a"], 0, "up_f_a"),
                           (np.full((h, w), 128, np.uint8), 0, "up_f_128")):
        out = torch.zeros(4 * ps, dtype=torch.uint8, device=gpu)
        _lib.check(lib.so_fme_planes(_plane(src, gpu).data_ptr(), h, w, wrap, out.data_ptr(), _lib.stream_handle()),
                   "so_fme_planes")
        torch.cuda.synchronize()
        o = out.cpu().numpy()
        F = np.zeros((2 * h - 1, 2 * w - 1), np.uint8)
        for a in (0, 1):
            for b in (0, 1):
                p = o[(2 * a + b) * ps:(2 * a + b) * ps + h * w].reshape(h, w)
                F[a::2, b::2] = p[: h - a, : w - b]
        assert (F == g[key]).all(), key


ME_GOPS = [
    ("gop_fme_vbs1", dict(qp=4, intra_dur=3, vbs=True, fme=True)),
    ("gop_fast_vbs1", dict(qp=4, intra_dur=4, vbs=True, fast_me=True)),
    ("gop_fast_fme", dict(qp=4, intra_dur=3, vbs=False, fast_me=True, fme=True)),
]


@pytest.mark.parametrize("name,cfg", ME_GOPS)
def test_gop_me_variants_golden(gpu, name, cfg, tmp_path, monkeypatch):
    from streamoptima_amd.Encoder import Y_Video_codec
    g = golden(name + ".npz")
    frames = g["frames"]
    f, h, w = frames.shape
    monkeypatch.chdir(tmp_path)
    enc = Y_Video_codec(h, w, f, 16, 16, cfg["qp"], cfg["intra_dur"], 0, 0.015, cfg["vbs"], nRefFrames=1,
                        y_only_frame_arr=frames, fast_me=cfg.get("fast_me", False), FMEEnable=cfg.get("fme", False),
                        device=gpu)
    psnr = enc.encode(block_size=16)
    assert np.allclose(psnr, g["psnr"], rtol=0, atol=1e-9), (psnr, g["psnr"])
    for i in range(f):
        _assert_frame(_sym_host(enc._symbols[i]), {"split": g[f"split{i}"], "mv": g[f"mv{i}"], "qtc": g[f"qtc{i}"],
                                                   "tokens": g[f"tokens{i}"], "recon": g["recon"][i]})
        assert (enc.decoded_device[i].cpu().numpy() == g["decoded"][i]).all()
    import gzip
    js = json.load(gzip.open(os.path.join(GOLDEN, name + "_bitstream.json.gz"), "rt"))
    pkg = enc.encoded_package
    for i in range(f):
        ft = pkg["frame_type_seq"][i]
        line = f"{ft}|" + enc.differential_encoder_frame(ft, pkg["MVS per Frame"][i], pkg["Qp_per_row_per_frame"][i])
        assert line == js["mv_lines"][i]


ME_VAR_CASES = [
    # (h, w, bs, sr, vbs, nref, me_mode, fme, wrap, kind)
    (64, 64, 16, 16, True, 2, 0, True, True, "tie"),
    (48, 80, 16, 16, False, 1, 0, True, False, "synth"),
    (64, 64, 8, 6, False, 1, 0, True, True, "synth"),      # bs 8 FME: generic kernel
    (16, 32, 16, 16, True, 1, 0, True, True, "synth"),     # no valid FME candidate: 128 prediction
    (256, 272, 16, 16, True, 1, 0, True, True, "synth"),   # several FME tiles
    (64, 96, 16, 16, True, 3, 1, False, True, "tie"),
    (64, 48, 8, 16, False, 2, 1, False, True, "synth"),    # bs 8 fast chain, two refs
    (96, 128, 16, 16, True, 2, 1, True, True, "synth"),
    (80, 64, 16, 16, False, 1, 2, False, True, "synth"),
    (80, 64, 8, 16, False, 1, 2, True, True, "tie"),
]


@pytest.mark.parametrize("h,w,bs,sr,vbs,nref,me_mode,fme,wrap,kind", ME_VAR_CASES)
def test_inter_me_variants_vs_oracle(gpu, h, w, bs, sr, vbs, nref, me_mode, fme, wrap, kind):
    from oracle import oracle as O
    from streamoptima_amd.engine import Engine
    seq = _frames(kind, h, w, 5 + h + 3 * w, n=nref + 1)
    cur, refs = seq[nref], [seq[k] for k in range(nref)]
    exp = O.inter_frame(cur, refs, bs, sr, 3, None, vbs, 0.015, me_mode=me_mode, fme=fme, fme_wrap=wrap)
    eng = Engine(h, w, bs, sr, vbs, 0.015, gpu, me_mode=me_mode, fme=fme)
    rp = [_plane(r, gpu) for r in refs]
    sym = eng.encode_p(_plane(cur, gpu), rp, 3, fme_wrap=wrap)
    torch.cuda.synchronize()
    hs = _sym_host(sym)
    _assert_frame(hs, exp)
    assert (hs["mae_num"] == exp["mae_num"]).all()
    if fme:
        rec = eng.recon_inter(rp, sym.split, sym.mv, sym.qtc, 3, fme_wrap=wrap)
        torch.cuda.synchronize()
        assert (rec.cpu().numpy() == O.inter_recon(refs, exp["split"], exp["mv"], exp["qtc"], bs, 3, fme=True,
                                                   fme_wrap=wrap)).all()


@pytest.mark.parametrize("name,cfg", GOPS[:2] + ME_GOPS[:2])
def test_decode_bitstream_reference_lines(gpu, name, cfg, tmp_path):
    """decoder.decode_bitstream (decoder.py:686-709) on the REFERENCE's text lines: host
    parse, GPU reconstruction == the reference's decoded frames."""
    import gzip
    from streamoptima_amd.decoder import decoder
    g = golden(name + ".npz")
    f, h, w = g["frames"].shape
    js = json.load(gzip.open(os.path.join(GOLDEN, name + "_bitstream.json.gz"), "rt"))
    mv_f, res_f = tmp_path / "mv.txt", tmp_path / "res.txt"
    mv_f.write_text("\n".join(js["mv_lines"]) + "\n")
    res_f.write_text("\n".join(js["residual_lines"]) + "\n")
    dec = decoder(0, cfg["intra_dur"], 16, f, h, w, cfg["qp"], 1, cfg.get("fme", False), 0.015, cfg["vbs"],
                  RCFlag=cfg.get("rc"), device=gpu)
    out = dec.decode_bitstream(str(mv_f), str(res_f))
    for i in range(f):
        assert (out[i] == g["decoded"][i]).all(), i


def test_transmit_then_decode_bitstream(gpu, tmp_path, monkeypatch):
    """encode -> transmit_bitstream -> decode_bitstream reproduces the encoder's recon."""
    from streamoptima_amd.Encoder import Y_Video_codec
    from streamoptima_amd.decoder import decoder
    from streamoptima_amd.synth import synth_sequence
    monkeypatch.chdir(tmp_path)
    seq = synth_sequence(4, 96, 128, seed=21)
    tables = json.load(open(os.path.join(GOLDEN, "rc_schedule.json")))["tables"]
    enc = Y_Video_codec(96, 128, 4, 16, 16, 4, 3, 0, 0.015, True, y_only_frame_arr=seq, RCFlag=1,
                        targetBR="2 mbps", qp_rate_tables=tables, device=gpu)
    enc.encode()
    enc.transmit_bitstream(mv_file=str(tmp_path / "mv.txt"), residual_file=str(tmp_path / "res.txt"))
    dec = decoder(0, 3, 16, 4, 96, 128, 4, 1, False, 0.015, True, RCFlag=1, targetBR="2 mbps",
                  qp_rate_tables=tables, device=gpu)
    out = dec.decode_bitstream(str(tmp_path / "mv.txt"), str(tmp_path / "res.txt"))
    for i in range(4):
        assert (out[i] == enc._symbols[i].recon.cpu().numpy()).all(), i


# ---------------------------------------------------------------- ROI and two-pass RC (configs[4])
# Build extension: no reference counterpart -- parity against the C oracle's
# restatement (oracle/gop.py encode_gop rc=3 / roi, oracle oc_qp_map).
def test_qp_map_kernel_vs_oracle(gpu):
    from oracle import oracle as O
    from streamoptima_amd.engine import Engine
    eng = Engine(96, 160, 16, 16, False, 0.015, gpu)
    rng = np.random.default_rng(5)
    tok = rng.integers(1, 400, size=eng.nb).astype(np.int32)
    roi = rng.integers(-3, 3, size=eng.nb).astype(np.int32)
    qr = rng.integers(0, 8, size=eng.nby).astype(np.int32)
    out = torch.full((eng.nb,), -7, dtype=torch.int32, device=gpu)
    for t, r, q in ((tok, roi, qr), (tok, None, None), (None, roi, qr)):
        eng.qp_map(_dev(t, gpu) if t is not None else None, 4, _dev(q, gpu) if q is not None else None,
                   _dev(r, gpu) if r is not None else None, out, qp_lo=1, qp_hi=9)
        torch.cuda.synchronize()
        assert (out.cpu().numpy() == O.qp_map(t, eng.nbx, eng.nby, 4, q, r, 1, 9)).all()
    # stripe rows only: rows outside [2, 4) keep their previous values
    out.fill_(-7)
    eng.qp_map(_dev(tok[2 * eng.nbx:4 * eng.nbx], gpu), 4, None, None, out, 2, 4)
    torch.cuda.synchronize()
    o = out.cpu().numpy().reshape(eng.nby, eng.nbx)
    assert (o[:2] == -7).all() and (o[4:] == -7).all()
    assert (o[2:4].reshape(-1) == O.qp_map(tok[2 * eng.nbx:4 * eng.nbx], eng.nbx, 2, 4)).all()


RC_GOPS = [
    # (name, vbs, rc, roi, fast, fme)
    ("two_pass_vbs", True, 3, False, False, False),
    ("two_pass_roi", False, 3, True, False, False),
    ("roi_rc1", True, 1, True, False, False),
    ("roi_only_fme", False, None, True, False, True),
    ("two_pass_fast", True, 3, True, True, False),
]


@pytest.mark.parametrize("name,vbs,rc,roi,fast,fme", RC_GOPS)
def test_gop_two_pass_roi_vs_oracle(gpu, name, vbs, rc, roi, fast, fme, tmp_path, monkeypatch):
    from oracle.gop import encode_gop
    from streamoptima_amd.Encoder import Y_Video_codec
    from streamoptima_amd.synth import synth_sequence
    monkeypatch.chdir(tmp_path)
    h, w, f = 96, 128, 5
    seq = synth_sequence(f, h, w, seed=31)
    # mixed complexity (two-pass needs blocks far from their row's mean): a smooth ramp on
    # the left quarter, a flat patch, texture elsewhere
    seq[:, :, : w // 4] = (np.arange(w // 4)[None, None, :] * 3 + np.arange(h)[None, :, None]).astype(np.uint8)
    seq[:, 32:64, 64:96] = 90
    tables = json.load(open(os.path.join(GOLDEN, "rc_schedule.json")))["tables"]
    roi_map = None
    if roi:
        roi_map = np.zeros((h // 16, w // 16), np.int32)
        roi_map[2:5, 2:6] = -2
        roi_map[0] = 2
    kw = dict(RCFlag=rc, targetBR="200 kbps" if rc else None, qp_rate_tables=tables if rc else None,
              intra_thresh=10 ** 9 if rc and rc > 1 else None)
    enc = Y_Video_codec(h, w, f, 16, 16, 4, 3, 0, 0.015, vbs, y_only_frame_arr=seq, fast_me=fast, FMEEnable=fme,
                        roi=roi_map, device=gpu, **kw)
    psnr = enc.encode()
    exp = encode_gop(seq, 4, 3, vbs=vbs, rc=rc, target=kw["targetBR"], tables=tables,
                     intra_thresh=kw["intra_thresh"], fast_me=fast, fme=fme,
                     roi=roi_map.reshape(-1) if roi else None)
    pkg = enc.encoded_package
    for i in range(f):
        _assert_frame(_sym_host(enc._symbols[i]), exp[i])
        assert (pkg["QP map per frame"][i] == exp[i]["qp_map"]).all()
        assert psnr[i] == exp[i]["psnr"]
        assert (enc.decoded_device[i].cpu().numpy() == exp[i]["recon"]).all()
    if rc == 3:   # the map really moved QPs (two-pass is not a no-op on this content)
        assert any(len(np.unique(pkg["QP map per frame"][i])) > 2 for i in range(f))


def test_two_pass_roi_bitstream_round_trip(gpu, tmp_path, monkeypatch):
    """RCFlag 3 + ROI: transmit_bitstream (+ the QP-map line) -> decode_bitstream == recon."""
    from streamoptima_amd.Encoder import Y_Video_codec
    from streamoptima_amd.decoder import decoder
    from streamoptima_amd.synth import synth_sequence
    monkeypatch.chdir(tmp_path)
    h, w, f = 96, 128, 4
    seq = synth_sequence(f, h, w, seed=8)
    seq[:, :, :48] = 60
    tables = json.load(open(os.path.join(GOLDEN, "rc_schedule.json")))["tables"]
    roi = [(32, 16, 96, 64, -2)]
    enc = Y_Video_codec(h, w, f, 16, 16, 4, 2, 0, 0.015, True, y_only_frame_arr=seq, RCFlag=3, targetBR="200 kbps",
                        qp_rate_tables=tables, intra_thresh=10 ** 9, roi=roi, device=gpu)
    enc.encode()
    files = [str(tmp_path / n) for n in ("mv.txt", "res.txt", "qp.txt")]
    enc.transmit_bitstream(mv_file=files[0], residual_file=files[1], qp_map_file=files[2])
    dec = decoder(0, 2, 16, f, h, w, 4, 1, False, 0.015, True, RCFlag=3, targetBR="200 kbps", qp_rate_tables=tables,
                  device=gpu)
    out = dec.decode_bitstream(files[0], files[1], qp_map_file=files[2])
    for i in range(f):
        assert (out[i] == enc._symbols[i].recon.cpu().numpy()).all(), i


# ---------------------------------------------------------------- persistent P-frame runs
@pytest.mark.parametrize("h,w,n,qp,seed", [(1088, 1920, 6, 4, 3), (2160, 3840, 4, 4, 0), (256, 384, 9, 2, 5),
                                             (208, 256, 33, 4, 7)])
def test_p_run_matches_per_frame(gpu, h, w, n, qp, seed):
    """so_encode_p_run (one persistent launch; frame i+1's tiles start while frame i's last
    rows finish) produces exactly the symbols of so_encode_p_frame called frame by frame,
    incl. a run longer than one launch's 32 frames, and no dependency wait times out."""
    from streamoptima_amd.engine import Engine, alloc_planes
    from streamoptima_amd.synth import synth_sequence_torch
    dev = gpu
    fr = alloc_planes(n + 1, h, w, dev)
    fr.copy_(synth_sequence_torch(n + 1, h, w, seed, dev))
    eng = Engine(h, w, 16, 16, False, 0.015, dev)
    i0 = eng.encode_i(fr[0], qp)
    ref_syms = []
    ref = i0.recon
    for k in range(1, n + 1):
        s = eng.encode_p(fr[k], [ref], qp)
        ref_syms.append(s)
        ref = s.recon
    outs = [eng.new_symbols(1) for _ in range(n)]
    eng.encode_p_run([fr[k] for k in range(1, n + 1)], i0.recon, qp, outs)
    torch.cuda.synchronize()
    assert not eng.run_timed_out()
    for k in range(n):
        a, b = _sym_host(outs[k]), _sym_host(ref_syms[k])
        _assert_frame(a, b, keys=("split", "mv", "qtc", "tokens", "recon"))
        assert torch.equal(outs[k].mae_num, ref_syms[k].mae_num)
        assert torch.equal(outs[k].sse, ref_syms[k].sse)
