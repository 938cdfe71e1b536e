"""Generate the golden vectors in tests/golden/ by running the REFERENCE encoder.

Run in the development container only (it needs /root/reference, which does not exist
on the GPU box):   python tests/golden/make_golden.py [--large]

What it does:
  * injects a stub `skimage.metrics` (PSNR = 10*log10(255^2/MSE) in float64, SSIM=NaN),
    forces the matplotlib Agg backend and imports /root/reference/Encoder.py;
  * runs the reference's own functions on deterministic synthetic input
    (streamoptima_amd/synth.py) from a scratch cwd (the reference writes files/ yuv/);
  * converts its outputs into the canonical array layout used by the oracle and the
    HIP path (see `canon_inter` / `canon_intra` below) and stores them as .npz / .json.

Only inputs and the reference's outputs are stored here: no reference source.
"""
from __future__ import annotations

import argparse
import contextlib
import hashlib
import io
import json
import os
import sys
import tempfile
import time
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from streamoptima_amd.synth import synth_sequence, tie_heavy_sequence  # noqa: E402


def import_reference():
    import matplotlib
    matplotlib.use("Agg")
    sk = types.ModuleType("skimage")
    skm = types.ModuleType("skimage.metrics")

    def psnr(a, b, data_range=None):
        a = np.asarray(a, dtype=np.float64)
        b = np.asarray(b, dtype=np.float64)
        return 10 * np.log10((255.0 ** 2) / np.mean((a - b) ** 2, dtype=np.float64))

    skm.peak_signal_noise_ratio = psnr
    skm.structural_similarity = lambda *a, **k: float("nan")
    sk.metrics = skm
    sys.modules["skimage"] = sk
    sys.modules["skimage.metrics"] = skm
    sys.path.insert(0, "/root/reference")
    import Encoder  # noqa: F401
    import decoder  # noqa: F401
    return sys.modules["Encoder"], sys.modules["decoder"]


class _NpCanvasProxy:
    """Forward to numpy, but make the hard-coded intra canvas ones((288,352))
    (Encoder.py:1165, 1248) frame-sized: SURVEY.md Appendix B.5 / C."""

    def __init__(self, h, w):
        self._h, self._w = h, w

    def __getattr__(self, name):
        return getattr(np, name)

    def ones(self, shape, *a, **k):
        if tuple(shape) == (288, 352):
            shape = (self._h, self._w)
        return np.ones(shape, *a, **k)


@contextlib.contextmanager
def canvas_patch(Encoder, h, w):
    old = Encoder.np
    Encoder.np = _NpCanvasProxy(h, w)
    try:
        yield
    finally:
        Encoder.np = old


def make_codec(Encoder, frames_arr, qp, vbs=False, lam=0.015, rc=None, target=None,
               tables=None, intra_thresh=None, intra_dur=None, nref=1, sr=16, bs=16,
               fast_me=False, fme=False, parallel_mode=0):
    f, h, w = frames_arr.shape
    return Encoder.Y_Video_codec(h, w, f, bs, sr, qp, intra_dur or f, 0, lam, vbs,
                                 nRefFrames=nref, y_only_frame_arr=frames_arr,
                                 fast_me=fast_me, FMEEnable=fme, RCFlag=rc,
                                 targetBR=target, frame_rate=30, qp_rate_tables=tables,
                                 intra_thresh=intra_thresh, ParallelMode=parallel_mode)


def canon_inter(mvs, qblocks, bs):
    nb = len(mvs)
    split = np.zeros(nb, np.uint8)
    mv = np.zeros((nb, 4, 3), np.int16)
    qtc = np.zeros((nb, bs * bs), np.int16)
    for i, (m, q) in enumerate(zip(mvs, qblocks)):
        assert m[0] == q[0]
        if m[0] == 0:
            mv[i, 0] = m[1]
            qtc[i] = np.asarray(q[1]).reshape(-1)
        else:
            split[i] = 1
            for j in range(4):
                mv[i, j] = m[1][j]
                qtc[i, j * (bs * bs // 4):(j + 1) * (bs * bs // 4)] = np.asarray(q[1][j]).reshape(-1)
    return split, mv, qtc


def canon_intra(mvs, qblocks, bs):
    nb = len(mvs)
    split = np.zeros(nb, np.uint8)
    mv = np.zeros((nb, 4), np.int16)
    qtc = np.zeros((nb, bs * bs), np.int16)
    for i, (m, q) in enumerate(zip(mvs, qblocks)):
        assert m[0] == q[0]
        if m[0] == 0:
            mv[i, 0] = m[1]
            qtc[i] = np.asarray(q[1]).reshape(-1)
        else:
            split[i] = 1
            for j in range(4):
                mv[i, j] = m[1][j]
                qtc[i, j * (bs * bs // 4):(j + 1) * (bs * bs // 4)] = np.asarray(q[1][j]).reshape(-1)
    return split, mv, qtc


def block_tokens(enc, qblocks, bs):
    out = np.zeros(len(qblocks), np.int32)
    for i, q in enumerate(qblocks):
        if q[0] == 0:
            out[i] = len(enc.entropy_encoder_block(q[1], bs))
        else:
            out[i] = sum(len(enc.entropy_encoder_block(s, bs // 2)) for s in q[1])
    return out


def quiet():
    return contextlib.redirect_stdout(io.StringIO())


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


# --------------------------------------------------------------------------------------
def gen_dct(Encoder, out):
    """Golden vector 1: 2D DCT-II / DCT-III (apply_2d_dct / apply_2d_idct, Encoder.py:779-817)."""
    enc = make_codec(Encoder, np.zeros((1, 32, 32), np.uint8), 4)
    rng = np.random.default_rng(1234)
    res = {}
    for n in (16, 8):
        k = 1200
        blocks = rng.integers(-255, 256, size=(k, n, n)).astype(np.float64)
        # tie-heavy half: force the DC sum to be == n/2 (mod n) so DC lands on x.5
        for b in range(k // 2):
            s = int(blocks[b].sum())
            blocks[b, 0, 0] += (n // 2 - s) % n
        blocks = np.clip(blocks, -255, 255)
        from scipy.fftpack import dct, idct
        raw = np.stack([dct(dct(b, axis=0, norm="ortho"), axis=1, norm="ortho") for b in blocks])
        tc = np.stack([enc.apply_2d_dct(b) for b in blocks]).astype(np.int32)
        # IDCT inputs: dequantised coefficients QTC*Q for a few QPs
        qp = rng.integers(0, 7, size=k)
        deq = np.stack([enc.quantize_TC(tc[i], enc.generate_Q_matrix(n, int(qp[i]))) *
                        enc.generate_Q_matrix(n, int(qp[i])) for i in range(k)]).astype(np.int32)
        rawi = np.stack([idct(idct(d.astype(np.int64), axis=0, norm="ortho"), axis=1, norm="ortho")
                         for d in deq])
        idc = np.stack([enc.apply_2d_idct(d.astype(np.int64)) for d in deq]).astype(np.int32)
        nraw = 256  # raw float64 bit patterns only for a subset (they do not compress)
        res[f"in{n}"] = blocks.astype(np.int16)
        res[f"raw{n}"] = raw[:nraw].view(np.uint64)
        res[f"tc{n}"] = tc.astype(np.int16)
        res[f"qp{n}"] = qp.astype(np.int8)
        res[f"deq{n}"] = deq
        res[f"rawi{n}"] = rawi[:nraw].view(np.uint64)
        res[f"idct{n}"] = idc.astype(np.int16)
        # 1-D vectors as well (each axis pass on its own)
        v = rng.integers(-4080, 4081, size=(1000, n)).astype(np.float64)
        res[f"v{n}"] = v.astype(np.int16)
        res[f"v{n}_dct"] = dct(v, axis=1, norm="ortho").view(np.uint64)
        res[f"v{n}_idct"] = idct(v, axis=1, norm="ortho").view(np.uint64)
    # token counts (entropy_encoder_block, Encoder.py:1086-1131) incl. all-zero and dense
    q = rng.integers(-2, 3, size=(3000, 16, 16)) * (rng.random((3000, 16, 16)) < rng.random((3000, 1, 1)))
    q[0] = 0
    q[1] = 1
    res["tok_in16"] = q.astype(np.int16)
    res["tok16"] = np.array([len(enc.entropy_encoder_block(b, 16)) for b in q], np.int32)
    res["tok_list16_first"] = np.array(enc.entropy_encoder_block(q[5], 16), np.int32)
    q8 = q[:, :8, :8]
    res["tok_in8"] = q8.astype(np.int16)
    res["tok8"] = np.array([len(enc.entropy_encoder_block(b, 8)) for b in q8], np.int32)
    np.savez_compressed(os.path.join(out, "dct_tokens.npz"), **res)


def gen_me_tie(Encoder, out):
    """Golden vector 2: find_best_match on tie-heavy content (Encoder.py:678-717)."""
    seq = tie_heavy_sequence(2, 288, 352, seed=3)
    cur = seq[1].astype(np.float64)
    ref = seq[0]
    enc = make_codec(Encoder, seq, 4)
    res16 = np.zeros((18, 22, 4), np.int32)
    for by in range(18):
        for bx in range(22):
            (dx, dy, r), mae = enc.find_best_match(cur[by*16:by*16+16, bx*16:bx*16+16], [ref], bx*16, by*16, 16, 16)
            res16[by, bx] = (dx, dy, r, int(round(mae * 256)) if np.isfinite(mae) else -1)
    # 8x8 sub-blocks on a band of rows, two references
    ref2 = tie_heavy_sequence(1, 288, 352, seed=9)[0]
    res8 = np.zeros((12, 44, 4), np.int32)
    for sy in range(12):
        for sx in range(44):
            (dx, dy, r), mae = enc.find_best_match(cur[sy*8:sy*8+8, sx*8:sx*8+8], [ref, ref2], sx*8, sy*8, 8, 16)
            res8[sy, sx] = (dx, dy, r, int(round(mae * 64)) if np.isfinite(mae) else -1)
    np.savez_compressed(os.path.join(out, "me_tie.npz"), cur=seq[1], ref=ref, ref2=ref2,
                        best16=res16, best8=res8)


def gen_inter(Encoder, out, vbs, name, qp=4, rc=None, target=None, tables=None):
    """Golden vector 3: one CIF P-frame through complete_inter_flow (Encoder.py:1644)."""
    seq = synth_sequence(2, 288, 352, seed=0)
    enc = make_codec(Encoder, seq, qp, vbs=vbs, rc=rc, target=target, tables=tables)
    enc.set_Qp(qp)
    cur = enc.pad_hw(seq[1], 16, 128)
    t0 = time.time()
    with quiet():
        mvs, avg_mae, qb, qprow, recon, rsize, stats = enc.complete_inter_flow(cur, [seq[0]], 16, 16)
    dt = time.time() - t0
    split, mv, qtc = canon_inter(mvs, qb, 16)
    tok = block_tokens(enc, qb, 16)
    assert tok.sum() == rsize
    np.savez_compressed(os.path.join(out, name), cur=seq[1], ref=seq[0], split=split, mv=mv,
                        qtc=qtc, tokens=tok, recon=recon, avg_mae=np.float64(avg_mae),
                        qp_per_row=np.array(qprow, np.int32), residual_size=np.int64(rsize),
                        row_stats=np.array(stats, np.float64), seconds=np.float64(dt))
    return dt


def gen_intra(Encoder, out, vbs, name, qp=6, h=288, w=352, seed=0):
    """Golden vector 4: one I-frame through complete_intra_flow (Encoder.py:1582)."""
    seq = synth_sequence(1, h, w, seed=seed)
    enc = make_codec(Encoder, seq, qp, vbs=vbs)
    enc.set_Qp(qp)
    cur = enc.pad_hw(seq[0], 16, 128)
    with canvas_patch(Encoder, h, w), quiet():
        mvs, avg_mae, qb, qprow, recon, resid, rsize, stats = enc.complete_intra_flow(cur, 0, 16, 16)
    split, mv, qtc = canon_intra(mvs, qb, 16)
    tok = block_tokens(enc, qb, 16)
    assert tok.sum() == rsize
    np.savez_compressed(os.path.join(out, name), cur=seq[0], split=split, mv=mv, qtc=qtc,
                        tokens=tok, recon=recon, avg_mae=np.float64(avg_mae))


def gen_gop(Encoder, out, name, frames, intra_dur, qp, vbs, rc=None, target=None,
            tables=None, intra_thresh=None, h=288, w=352, seed=0, **kw):
    """Golden vector 5: encode() of a short GOP plus the text bitstream lines."""
    seq = synth_sequence(frames, h, w, seed=seed)
    enc = make_codec(Encoder, seq, qp, vbs=vbs, rc=rc, target=target, tables=tables,
                     intra_thresh=intra_thresh, intra_dur=intra_dur, **kw)
    with canvas_patch(Encoder, h, w), quiet():
        psnr = enc.encode(block_size=16)
    pkg = enc.encoded_package
    res = {"frames": seq, "psnr": np.array(psnr, np.float64),
           "frame_type": np.array(pkg["frame_type_seq"], np.int8),
           "mae": np.array(pkg["MAE per Frame"], np.float64)}
    lines_mv, lines_res = [], []
    for i in range(frames):
        ft = pkg["frame_type_seq"][i]
        mvs = pkg["MVS per Frame"][i]
        qb = pkg["approx residual"][i]
        if ft == 0:
            split, mv, qtc = canon_intra(mvs, qb, 16)
        else:
            split, mv, qtc = canon_inter(mvs, qb, 16)
        res[f"split{i}"], res[f"mv{i}"], res[f"qtc{i}"] = split, mv, qtc
        res[f"qp_per_row{i}"] = np.array(pkg["Qp_per_row_per_frame"][i], np.int32)
        res[f"tokens{i}"] = block_tokens(enc, qb, 16)
        lines_mv.append(f"{ft}|" + enc.differential_encoder_frame(ft, mvs, pkg["Qp_per_row_per_frame"][i]))
        lines_res.append(enc.entropy_encoder_frame(qb, 16))
    # the reference saves its reconstruction to yuv/y_only_reconstructed.yuv (Encoder.py:1894)
    recon = np.fromfile("yuv/y_only_reconstructed.yuv", np.uint8).reshape(frames, h, w)
    res["recon"] = recon
    dec = enc.decoder.decoded_vid
    res["decoded"] = np.stack(dec)
    np.savez_compressed(os.path.join(out, name + ".npz"), **res)
    import gzip
    with gzip.open(os.path.join(out, name + "_bitstream.json.gz"), "wt") as f:
        json.dump({"mv_lines": lines_mv, "residual_lines": lines_res}, f)


def gen_fme_frames(Encoder, out):
    """frac_me_reference_frame (Encoder.py:388-403) of a uint8 list (wrapping row sums) and
    of a list that still holds the float64 all-128 start frame (no wrap)."""
    rng = np.random.default_rng(77)
    a = rng.integers(0, 256, size=(24, 40)).astype(np.uint8)
    a[:4] = rng.integers(200, 256, size=(4, 40))         # row sums past 255
    b = rng.integers(0, 256, size=(24, 40)).astype(np.uint8)
    enc = make_codec(Encoder, np.zeros((1, 24, 40), np.uint8), 4)
    up_u8 = enc.frac_me_reference_frame([a, b], 16)
    up_f = enc.frac_me_reference_frame([np.ones((24, 40)) * 128, a], 16)
    for f in up_u8 + up_f:
        assert f.min() >= 0 and f.max() <= 255 and np.all(f == np.round(f))
    np.savez_compressed(os.path.join(out, "fme_frames.npz"), a=a, b=b,
                        up_u8_a=np.asarray(up_u8[0], np.uint8), up_u8_b=np.asarray(up_u8[1], np.uint8),
                        up_f_128=np.asarray(up_f[0], np.uint8), up_f_a=np.asarray(up_f[1], np.uint8))


def gen_inter_me_variants(Encoder, out):
    """complete_inter_flow with FMEEnable and/or fast_me (Encoder.py:462-585, 678-742,
    1644-1709), plus fast_me under ParallelMode 2 (inter_prediction_parallel :587-676)."""
    cases = [
        # name, h, w, sr, vbs, fast, fme, nref, parallel_mode
        ("fme_cif_vbs0", 288, 352, 16, False, False, True, 1, 0),
        ("fme_96x128_vbs1", 96, 128, 16, True, False, True, 1, 0),
        ("fme_64x96_sr4_vbs1", 64, 96, 4, True, False, True, 1, 0),
        ("fme_64x96_nref2", 64, 96, 8, True, False, True, 2, 0),
        ("fast_cif_vbs0", 288, 352, 16, False, True, False, 1, 0),
        ("fast_cif_vbs1", 288, 352, 16, True, True, False, 1, 0),
        ("fast_cif_nref2_vbs1", 288, 352, 16, True, True, False, 2, 0),
        ("fast_fme_cif_vbs1", 288, 352, 16, True, True, True, 1, 0),
        ("fast_par2_cif", 288, 352, 16, False, True, False, 2, 2),
    ]
    res = {}
    for name, h, w, sr, vbs, fast, fme, nref, pm in cases:
        seq = synth_sequence(3, h, w, seed=11)
        enc = make_codec(Encoder, seq, 4, vbs=vbs, sr=sr, fast_me=fast, fme=fme, nref=nref, parallel_mode=pm)
        enc.set_Qp(4)
        cur = enc.pad_hw(seq[2], 16, 128)
        refs = [seq[0], seq[1]][-nref:] if nref > 1 else [seq[1]]
        t0 = time.time()
        with quiet():
            mvs, avg_mae, qb, qprow, recon, rsize, stats = enc.complete_inter_flow(cur, list(refs), 16, sr)
        split, mv, qtc = canon_inter(mvs, qb, 16)
        tok = block_tokens(enc, qb, 16)
        assert tok.sum() == rsize
        for k, v in dict(split=split, mv=mv, qtc=qtc, tokens=tok, recon=recon).items():
            res[f"{name}__{k}"] = v
        res[f"{name}__avg_mae"] = np.float64(avg_mae)
        res[f"{name}__cur"] = seq[2]
        res[f"{name}__refs"] = np.stack(refs)
        res[f"{name}__cfg"] = np.array([h, w, sr, int(vbs), int(fast), int(fme), nref, pm], np.int32)
        print(f"  {name}: {time.time() - t0:.1f}s", flush=True)
    np.savez_compressed(os.path.join(out, "inter_me_variants.npz"), **res)


def canon_residuals(res_list, bs):
    """inter/intra_prediction's residual_per_block [(0, r bs x bs) | (1, [r x 4])] as
    int16 [nb][bs*bs] (split: the 4 sub-blocks' (bs/2)^2 values in Z order)."""
    out = np.zeros((len(res_list), bs * bs), np.int16)
    for i, (s, r) in enumerate(res_list):
        if s == 0:
            out[i] = np.asarray(r).reshape(-1)
        else:
            q = bs * bs // 4
            for j in range(4):
                out[i, j * q:(j + 1) * q] = np.asarray(r[j]).reshape(-1)
    return out


def gen_blockapi(Encoder, out):
    """The reference's per-block / per-frame public methods, called directly:
    inter_prediction (Encoder.py:462-585), intra_prediction (:1238-1347), find_best_match
    with FMEEnable on frac frames (:678-717), reconstruct_block (:824-827) and
    calculate_RD_cost (:1133-1158)."""
    res = {}
    rng = np.random.default_rng(4321)
    # inter_prediction, CIF, VBS on and off (mvs, average MAE, unquantised residuals)
    seq = synth_sequence(2, 288, 352, seed=0)
    for vbs in (False, True):
        enc = make_codec(Encoder, seq, 4, vbs=vbs)
        enc.set_Qp(4)
        cur = enc.pad_hw(seq[1], 16, 128)
        with quiet():
            mvs, avg, resid = enc.inter_prediction(cur, [seq[0]], 16, 16)
        split, mv, _ = canon_inter(mvs, [(m[0], np.zeros((16, 16)) if m[0] == 0 else [np.zeros((8, 8))] * 4)
                                         for m in mvs], 16)
        k = f"inter_vbs{int(vbs)}"
        res[k + "_split"], res[k + "_mv"] = split, mv
        res[k + "_avg_mae"] = np.float64(avg)
        res[k + "_resid"] = canon_residuals(resid, 16)
    res["inter_cur"], res["inter_ref"] = seq[1], seq[0]
    # inter_prediction with FMEEnable: complete_inter_flow's call (frac frames, 2 sr; :1647-1651)
    sq = synth_sequence(2, 64, 96, seed=4)
    enc = make_codec(Encoder, sq, 4, vbs=True, fme=True)
    enc.set_Qp(4)
    cur = enc.pad_hw(sq[1], 16, 128)
    frac = enc.frac_me_reference_frame([sq[0]], 16)
    with quiet():
        mvs, avg, resid = enc.inter_prediction(cur, frac, 16, 32)
    split, mv, _ = canon_inter(mvs, [(m[0], np.zeros((16, 16)) if m[0] == 0 else [np.zeros((8, 8))] * 4)
                                     for m in mvs], 16)
    res["fme_split"], res["fme_mv"], res["fme_avg_mae"] = split, mv, np.float64(avg)
    res["fme_resid"] = canon_residuals(resid, 16)
    res["fme_cur"], res["fme_ref"] = sq[1], sq[0]
    # find_best_match on the frac frame (FMEEnable), full blocks and 8x8 sub-blocks
    fbm = []
    for by in range(4):
        for bx in range(6):
            for bs_, off in ((16, (0, 0)), (8, (8, 8))):
                x, y = bx * 16 + off[0], by * 16 + off[1]
                (dx, dy, r), mae = enc.find_best_match(cur[y:y + bs_, x:x + bs_], frac, 2 * x, 2 * y, bs_, 32)
                fbm.append((x, y, bs_, dx, dy, r, int(mae * bs_ * bs_) if np.isfinite(mae) else -1))
    res["fme_fbm"] = np.array(fbm, np.int32)
    # intra_prediction, CIF, VBS on (canvas 288x352 is the frame here)
    sq = synth_sequence(1, 288, 352, seed=0)
    enc = make_codec(Encoder, sq, 6, vbs=True)
    enc.set_Qp(6)
    cur = enc.pad_hw(sq[0], 16, 128)
    with quiet():
        mvs, avg, resid, canvas = enc.intra_prediction(cur, 0, 16, 16)
    split, mv, _ = canon_intra(mvs, [(m[0], np.zeros((16, 16)) if m[0] == 0 else [np.zeros((8, 8))] * 4)
                                     for m in mvs], 16)
    res["intra_cur"], res["intra_split"], res["intra_mv"] = sq[0], split, mv
    res["intra_avg_mae"] = np.float64(avg)
    res["intra_resid"] = canon_residuals(resid, 16)
    res["intra_canvas"] = np.asarray(canvas, np.float64)
    # reconstruct_block: predicted uint8 + dequantised IDCT of QTC, Q of QP 0..6, both sizes
    enc = make_codec(Encoder, np.zeros((1, 32, 32), np.uint8), 4)
    for n in (16, 8):
        kb = 300
        pred = rng.integers(0, 256, size=(kb, n, n)).astype(np.uint8)
        qtc = (rng.integers(-6, 7, size=(kb, n, n)) * (rng.random((kb, n, n)) < 0.3)).astype(np.int64)
        qp = rng.integers(0, 7, size=kb)
        rec = np.stack([enc.reconstruct_block(pred[i], qtc[i], enc.generate_Q_matrix(n, int(qp[i])))
                        for i in range(kb)])
        res[f"rb{n}_pred"], res[f"rb{n}_qtc"], res[f"rb{n}_qp"] = pred, qtc.astype(np.int16), qp.astype(np.int8)
        res[f"rb{n}_out"] = rec.astype(np.uint8)
    # calculate_RD_cost: (frame_type, split) x residual blocks x QP, float64 costs
    cost, cin = [], []
    for i in range(200):
        ft, sp = int(rng.integers(0, 2)), int(rng.integers(0, 2))
        qp = int(rng.integers(0, 7))
        mae = float(rng.integers(0, 40 * 256)) / 256.0
        enc.set_Qp(qp)
        r16 = rng.integers(-60, 61, size=(16, 16)).astype(np.float64)
        resid = r16 if sp == 0 else [r16[:8, :8], r16[:8, 8:], r16[8:, :8], r16[8:, 8:]]
        cost.append(enc.calculate_RD_cost(ft, sp, mae, resid, 16, 8, 0.015))
        cin.append((ft, sp, qp, mae))
        res[f"rd_res{i}"] = r16.astype(np.int16)
    res["rd_in"] = np.array(cin, np.float64)
    res["rd_cost"] = np.array(cost, np.float64)
    np.savez_compressed(os.path.join(out, "blockapi.npz"), **res)


def gen_yuv(Encoder, out):
    """YUV file I/O (video_manager.py:4-241, Encoder.read_yuv :110-126): the reference's
    Video_Manager on a 21-frame CIF 4:2:0 file (its constructor always reads 21 frames) and
    read_yuv on the same file; sha256 of each output (the file is regenerated by the tests
    from streamoptima_amd/synth.py:write_synth_yuv420)."""
    import video_manager as vmod
    from streamoptima_amd.synth import write_synth_yuv420
    path = os.path.join(os.getcwd(), "cif.yuv")
    write_synth_yuv420(path, 21, 288, 352, seed=12)
    vm = vmod.Video_Manager(path, 288, 352, 21, "yuv_420")
    up = vm.upscale_yuv420_to_yuv444()
    rgb = vm.convert_yuv444_to_rgb()
    y = vm.extract_y_only()
    ry = Encoder.Y_Video_codec.read_yuv(path, 288, 352, 21)
    rec = {"frames": 21, "h": 288, "w": 352, "seed": 12,
           "yuv420_shape": list(vm.vid_frames_yuv420.shape), "yuv420_sha": sha(vm.vid_frames_yuv420),
           "upscale_shape": list(up.shape), "upscale_sha": sha(up),
           "yuv444_shape": list(vm.vid_frames_yuv444.shape), "yuv444_sha": sha(vm.vid_frames_yuv444),
           "rgb_shape": list(rgb.shape), "rgb_sha": sha(rgb), "rgb_dtype": str(rgb.dtype),
           "y_shape": list(y.shape), "y_sha": sha(y), "read_yuv_sha": sha(np.asarray(ry)),
           "read_yuv_dtype": str(np.asarray(ry).dtype)}
    with open(os.path.join(out, "yuv_io.json"), "w") as f:
        json.dump(rec, f, indent=1)


def gen_rc(Encoder, out):
    """Golden vector 6: the per-row QP schedule (Encoder.py:78-88, 1576-1609)."""
    tables = [[9000, 6000, 4000, 2600, 1700, 1100, 700, 450, 300, 200],
              [7000, 4500, 3000, 2000, 1300, 850, 550, 350, 230, 150]]
    cases = []
    for target in ["2 mbps", "1500 kbps", "900000 bps", "3 mbps"]:
        for h, w in [(288, 352), (1088, 1920)]:
            enc = make_codec(Encoder, np.zeros((1, h, w), np.uint8), 4, rc=1, target=target,
                             tables=tables)
            budget = enc.bitrate_per_row
            qps, spent = [], 0
            for r in range(h // 16):
                if r == 0:
                    budget = enc.bitrate_per_row
                else:
                    budget = enc.bitrate_per_row + (budget - spent)
                got = enc.get_appropriate_Qp_value(0, budget)
                if got is None:
                    qps.append(None)
                    break
                q, spent = got
                qps.append(q)
            cases.append({"target": target, "h": h, "w": w, "bitrate_per_row": enc.bitrate_per_row,
                          "qps": qps})
    with open(os.path.join(out, "rc_schedule.json"), "w") as f:
        json.dump({"tables": tables, "cases": cases}, f, indent=1)
    return tables


def gen_large(Encoder, out):
    """Golden vector 7: 2-frame I+P encodes at 1920x1088 and 3840x2160 as sha256."""
    res = {}
    for (h, w, seed) in [(1088, 1920, 0), (2160, 3840, 0)]:
        seq = synth_sequence(2, h, w, seed=seed)
        enc = make_codec(Encoder, seq, 4, intra_dur=2)
        t0 = time.time()
        with canvas_patch(Encoder, h, w), quiet():
            psnr = enc.encode(block_size=16)
        dt = time.time() - t0
        pkg = enc.encoded_package
        recon = np.fromfile("yuv/y_only_reconstructed.yuv", np.uint8).reshape(2, h, w)
        entry = {"seconds": dt, "psnr": list(map(float, psnr)),
                 "frame_type": list(pkg["frame_type_seq"]), "mae": list(map(float, pkg["MAE per Frame"]))}
        for i in range(2):
            mvs, qb = pkg["MVS per Frame"][i], pkg["approx residual"][i]
            if pkg["frame_type_seq"][i] == 0:
                split, mv, qtc = canon_intra(mvs, qb, 16)
            else:
                split, mv, qtc = canon_inter(mvs, qb, 16)
            entry[f"split{i}"] = sha(split)
            entry[f"mv{i}"] = sha(mv)
            entry[f"qtc{i}"] = sha(qtc)
            entry[f"tokens{i}"] = int(block_tokens(enc, qb, 16).sum())
            entry[f"recon{i}"] = sha(recon[i])
        res[f"{w}x{h}"] = entry
        print(f"large {w}x{h}: {dt:.1f}s", flush=True)
    with open(os.path.join(out, "large_hashes.json"), "w") as f:
        json.dump(res, f, indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--large", action="store_true", help="also the 1088p/4K hashes (~10 min)")
    ap.add_argument("--only", default=None)
    args = ap.parse_args()
    out = HERE
    Encoder, _ = import_reference()
    scratch = tempfile.mkdtemp(prefix="so_golden_")
    os.makedirs(os.path.join(scratch, "files"))
    os.makedirs(os.path.join(scratch, "yuv"))
    os.chdir(scratch)
    todo = args.only.split(",") if args.only else ["dct", "me", "inter", "intra", "rc", "gop"]
    if "dct" in todo:
        gen_dct(Encoder, out); print("dct done", flush=True)
    if "me" in todo:
        gen_me_tie(Encoder, out); print("me done", flush=True)
    tables = gen_rc(Encoder, out) if "rc" in todo or "gop" in todo else None
    if "inter" in todo:
        print("inter vbs0", gen_inter(Encoder, out, False, "cif_p_vbs0.npz"), flush=True)
        print("inter vbs1", gen_inter(Encoder, out, True, "cif_p_vbs1.npz"), flush=True)
        print("inter rc", gen_inter(Encoder, out, True, "cif_p_vbs1_rc.npz", rc=1,
                                    target="2 mbps", tables=tables), flush=True)
    if "intra" in todo:
        gen_intra(Encoder, out, False, "cif_i_qp6_vbs0.npz")
        gen_intra(Encoder, out, True, "cif_i_qp6_vbs1.npz")
        gen_intra(Encoder, out, True, "i_64x128_vbs1.npz", qp=3, h=64, w=128, seed=5)
        print("intra done", flush=True)
    if "gop" in todo:
        gen_gop(Encoder, out, "gop_cif_vbs0", frames=4, intra_dur=4, qp=4, vbs=False)
        print("gop0 done", flush=True)
        gen_gop(Encoder, out, "gop_cif_vbs1_rc1", frames=3, intra_dur=3, qp=4, vbs=True, rc=1,
                target="2 mbps", tables=tables)
        print("gop1 done", flush=True)
        gen_gop(Encoder, out, "gop_small_rc2", frames=4, intra_dur=4, qp=3, vbs=True, rc=2,
                target="1 mbps", tables=tables, intra_thresh=150, h=64, w=128, seed=7)
        print("gop2 done", flush=True)
    if "fme" in todo:
        gen_fme_frames(Encoder, out)
        gen_inter_me_variants(Encoder, out)
        print("fme/fast frames done", flush=True)
    if "gopme" in todo:
        gen_gop(Encoder, out, "gop_fme_vbs1", frames=3, intra_dur=3, qp=4, vbs=True, h=64, w=96, seed=4,
                fme=True)
        # (no nRefFrames > 1 GOP: the reference's closed-loop decode resets its reference
        # list at every I-frame, decoder.py:520, and then indexes a missing reference,
        # IndexError at decoder.py:117; the float-start no-wrap frac frame is pinned by
        # fme_frames.npz instead)
        gen_gop(Encoder, out, "gop_fast_vbs1", frames=4, intra_dur=4, qp=4, vbs=True, h=96, w=128, seed=6,
                fast_me=True)
        gen_gop(Encoder, out, "gop_fast_fme", frames=3, intra_dur=3, qp=4, vbs=False, h=64, w=96, seed=8,
                fast_me=True, fme=True)
        print("gop fme/fast done", flush=True)
    if "yuv" in todo:
        gen_yuv(Encoder, out)
        print("yuv done", flush=True)
    if "blockapi" in todo:
        gen_blockapi(Encoder, out)
        print("blockapi done", flush=True)
    if args.large:
        gen_large(Encoder, out)


if __name__ == "__main__":
    main()
