"""The drop-in per-block public methods of Y_Video_codec (streamoptima_amd/blockapi.py) on
the GPU, each against the reference's own outputs (tests/golden/, make_golden.py)."""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def _codec(gpu, h=288, w=352, qp=4, vbs=False, fme=False, rc=None, **kw):
    from streamoptima_amd.Encoder import Y_Video_codec
    c = Y_Video_codec(h, w, 2, 16, 16, qp, 2, 0, 0.015, vbs, FMEEnable=fme, RCFlag=rc, device=gpu, **kw)
    c.set_Qp(qp)
    return c


def _canon(mvs, nb):
    split = np.zeros(nb, np.uint8)
    mv = np.zeros((nb, 4, 3), np.int16)
    for i, m in enumerate(mvs):
        if m[0] == 0:
            mv[i, 0] = m[1]
        else:
            split[i] = 1
            for j in range(4):
                mv[i, j] = m[1][j]
    return split, mv


def _canon_res(res, bs=16):
    out = np.zeros((len(res), bs * bs), np.int64)
    for i, (s, r) in enumerate(res):
        out[i] = np.asarray(r).reshape(-1) if s == 0 else np.concatenate([np.asarray(x).reshape(-1) for x in r])
    return out


def test_find_best_match_tie_golden(gpu):
    """find_best_match (Encoder.py:678-717) per block, 16x16 one reference and 8x8 two
    references, on tie-heavy content: golden me_tie.npz."""
    g = golden("me_tie.npz")
    c = _codec(gpu)
    cur = g["cur"].astype(np.float64)
    for by in range(0, 18, 2):
        for bx in range(0, 22, 3):
            (dx, dy, r), mae = c.find_best_match(cur[by * 16:by * 16 + 16, bx * 16:bx * 16 + 16], [g["ref"]], bx * 16,
                                                 by * 16, 16, 16)
            assert (dx, dy, r, int(round(mae * 256))) == tuple(g["best16"][by, bx]), (by, bx)
    for sy in range(0, 12, 3):
        for sx in range(0, 44, 5):
            (dx, dy, r), mae = c.find_best_match(cur[sy * 8:sy * 8 + 8, sx * 8:sx * 8 + 8], [g["ref"], g["ref2"]], sx * 8,
                                                 sy * 8, 8, 16)
            assert (dx, dy, r, int(round(mae * 64))) == tuple(g["best8"][sy, sx]), (sy, sx)


def test_find_best_match_fme_golden(gpu):
    """find_best_match with FMEEnable on the frac frame at doubled coordinates and range."""
    g = golden("blockapi.npz")
    c = _codec(gpu, 64, 96, vbs=True, fme=True)
    cur = c.pad_hw(g["fme_cur"], 16, 128)
    frac = c.frac_me_reference_frame([g["fme_ref"]], 16)
    for x, y, bs, dx, dy, r, mae_n in g["fme_fbm"]:
        (gdx, gdy, gr), mae = c.find_best_match(cur[y:y + bs, x:x + bs], frac, 2 * x, 2 * y, bs, 32)
        assert (gdx, gdy, gr) == (dx, dy, r), (x, y, bs)
        assert (int(mae * bs * bs) if np.isfinite(mae) else -1) == mae_n


@pytest.mark.parametrize("vbs", [False, True])
def test_inter_prediction_golden(gpu, vbs):
    g = golden("blockapi.npz")
    k = f"inter_vbs{int(vbs)}"
    c = _codec(gpu, vbs=vbs)
    cur = c.pad_hw(g["inter_cur"], 16, 128)
    mvs, avg, res = c.inter_prediction(cur, [g["inter_ref"]], 16, 16)
    split, mv = _canon(mvs, len(mvs))
    assert (split == g[k + "_split"]).all() and (mv == g[k + "_mv"]).all()
    assert avg == float(g[k + "_avg_mae"])
    assert (_canon_res(res) == g[k + "_resid"]).all()


def test_inter_prediction_fme_golden(gpu):
    """complete_inter_flow's FME call: frac frames and 2 x sr (Encoder.py:1647-1651)."""
    g = golden("blockapi.npz")
    c = _codec(gpu, 64, 96, vbs=True, fme=True)
    cur = c.pad_hw(g["fme_cur"], 16, 128)
    frac = c.frac_me_reference_frame([g["fme_ref"]], 16)
    mvs, avg, res = c.inter_prediction(cur, frac, 16, 32)
    split, mv = _canon(mvs, len(mvs))
    assert (split == g["fme_split"]).all() and (mv == g["fme_mv"]).all()
    assert avg == float(g["fme_avg_mae"])
    assert (_canon_res(res) == g["fme_resid"]).all()


def test_intra_prediction_golden(gpu):
    g = golden("blockapi.npz")
    c = _codec(gpu, qp=6, vbs=True)
    cur = c.pad_hw(g["intra_cur"], 16, 128)
    mvs, avg, res, canvas = c.intra_prediction(cur, 0, 16, 16)
    nb = len(mvs)
    split = np.array([m[0] for m in mvs], np.uint8)
    mv = np.array([[m[1]] * 4 if m[0] == 0 else m[1] for m in mvs], np.int16)
    assert (split == g["intra_split"]).all()
    assert (mv[split == 1] == g["intra_mv"][split == 1]).all()
    assert (mv[split == 0, 0] == g["intra_mv"][split == 0, 0]).all()
    assert avg == float(g["intra_avg_mae"])
    assert (_canon_res(res) == g["intra_resid"]).all()
    assert np.array_equal(canvas, g["intra_canvas"]) and nb == 396


@pytest.mark.parametrize("n", [16, 8])
def test_apply_2d_dct_idct_golden(gpu, n):
    """apply_2d_dct / apply_2d_idct (Encoder.py:779-817) on 1,200 tie-heavy blocks each:
    one launch for the whole stack."""
    g = golden("dct_tokens.npz")
    c = _codec(gpu)
    assert (c.apply_2d_dct(g[f"in{n}"].astype(np.float64)) == g[f"tc{n}"]).all()
    assert (c.apply_2d_idct(g[f"deq{n}"].astype(np.float64)) == g[f"idct{n}"]).all()
    one = c.apply_2d_dct(g[f"in{n}"][0].astype(np.float64))        # the reference's one-block call
    assert one.shape == (n, n) and (one == g[f"tc{n}"][0]).all()


@pytest.mark.parametrize("n", [16, 8])
def test_reconstruct_block_golden(gpu, n):
    g = golden("blockapi.npz")
    c = _codec(gpu)
    for i in range(0, len(g[f"rb{n}_qp"]), 7):
        Q = c.generate_Q_matrix(n, int(g[f"rb{n}_qp"][i]))
        out = c.reconstruct_block(g[f"rb{n}_pred"][i], g[f"rb{n}_qtc"][i].astype(np.int64), Q)
        assert out.dtype == np.uint8 and (out == g[f"rb{n}_out"][i]).all(), i


def test_calculate_rd_cost_golden(gpu):
    g = golden("blockapi.npz")
    c = _codec(gpu)
    for i, (ft, sp, qp, mae) in enumerate(g["rd_in"]):
        c.set_Qp(int(qp))
        r = g[f"rd_res{i}"].astype(np.float64)
        res = r if sp == 0 else [r[:8, :8], r[:8, 8:], r[8:, :8], r[8:, 8:]]
        assert c.calculate_RD_cost(int(ft), int(sp), float(mae), res, 16, 8, 0.015) == g["rd_cost"][i], i


@pytest.mark.parametrize("name,vbs,rc", [("cif_p_vbs0.npz", False, None), ("cif_p_vbs1.npz", True, None),
                                         ("cif_p_vbs1_rc.npz", True, 1)])
def test_reconstruct_frame_golden(gpu, name, vbs, rc):
    """reconstruct_frame (Encoder.py:831-932) from the reference's own mvs / QTC lists."""
    from streamoptima_amd.package import frame_mvs, frame_residuals
    g = golden(name)
    c = _codec(gpu, vbs=vbs, rc=rc)
    host = {"frame_type": 1, "split": g["split"], "mv": g["mv"], "qtc": g["qtc"]}
    mvs, qb = frame_mvs(host, 16), frame_residuals(host, 16)
    rec = c.reconstruct_frame(mvs, [g["ref"]], qb, g["qp_per_row"].tolist(), 16)
    assert (rec == g["recon"]).all()


def test_calculate_metrics_golden(gpu):
    g = golden("gop_cif_vbs0.npz")
    c = _codec(gpu)
    for i in range(len(g["psnr"])):
        psnr, ssim = c.calculate_metrics(g["frames"][i], g["recon"][i])
        assert psnr == pytest.approx(float(g["psnr"][i]), abs=1e-9) and np.isnan(ssim)


def test_frac_me_reference_frame_golden(gpu):
    g = golden("fme_frames.npz")
    c = _codec(gpu, 24, 40, fme=True)
    up = c.frac_me_reference_frame([g["a"], g["b"]], 16)
    assert (up[0] == g["up_u8_a"]).all() and (up[1] == g["up_u8_b"]).all() and up[0].dtype == np.float64
    up = c.frac_me_reference_frame([np.ones((24, 40)) * 128, g["a"]], 16)
    assert (up[0] == g["up_f_128"]).all() and (up[1] == g["up_f_a"]).all()

