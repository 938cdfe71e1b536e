"""Host-side logic (no GPU): rate-control schedule, text bitstream, package building,
synthetic input, the numpy CPU-baseline port."""
import gzip
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden


def _codec(h, w, **kw):
    from streamoptima_amd.Encoder import Y_Video_codec
    return Y_Video_codec(h, w, 1, 16, 16, 4, 1, 0, 0.015, False, y_only_frame_arr=np.zeros((1, h, w), np.uint8),
                         **kw)


def test_rc_schedule_matches_reference():
    js = json.load(open(os.path.join(GOLDEN, "rc_schedule.json")))
    for case in js["cases"]:
        enc = _codec(case["h"], case["w"], RCFlag=1, targetBR=case["target"], qp_rate_tables=js["tables"])
        assert enc.bitrate_per_row == case["bitrate_per_row"]
        if None in case["qps"]:
            with pytest.raises(TypeError):
                enc.row_qp_schedule(case["h"] // 16)
        else:
            assert enc.row_qp_schedule(case["h"] // 16) == case["qps"]


def test_target_bitrate_units():
    assert _codec(32, 32, targetBR="3 kbps").target_bitrate == 3 * 1024
    assert _codec(32, 32, targetBR="2 mbps").target_bitrate == 2 * 1048576
    assert _codec(32, 32, targetBR="777 bps").target_bitrate == 777


def test_q_matrix_and_set_qp():
    enc = _codec(32, 32)
    q = enc.generate_Q_matrix(4, 2)
    assert q.tolist() == [[4, 4, 4, 8], [4, 4, 8, 16], [4, 8, 16, 16], [8, 16, 16, 16]]
    enc.set_Qp(0)
    assert enc.Qpm1 == 0 and enc.Qm1.shape == (8, 8)


@pytest.mark.parametrize("name,rc", [("gop_cif_vbs0", None), ("gop_cif_vbs1_rc1", 1), ("gop_small_rc2", 2)])
def test_bitstream_text_matches_reference(name, rc):
    from streamoptima_amd.bitstream import differential_encoder_frame, entropy_encoder_frame
    from streamoptima_amd.package import frame_mvs, frame_residuals
    js = json.load(gzip.open(os.path.join(GOLDEN, name + "_bitstream.json.gz"), "rt"))
    g = golden(name + ".npz")
    w = g["frames"].shape[2]
    for i, ft in enumerate(g["frame_type"].tolist()):
        host = {"frame_type": ft, "split": g[f"split{i}"], "mv": g[f"mv{i}"], "qtc": g[f"qtc{i}"]}
        line = f"{ft}|" + differential_encoder_frame(ft, frame_mvs(host, 16), g[f"qp_per_row{i}"].tolist(), rc, w / 16)
        assert line == js["mv_lines"][i]
        assert entropy_encoder_frame(frame_residuals(host, 16), 16) == js["residual_lines"][i]


def test_entropy_block_and_token_count():
    from streamoptima_amd.bitstream import entropy_encoder_block, token_count
    g = golden("dct_tokens.npz")
    for b, t in zip(g["tok_in16"][:500], g["tok16"][:500]):
        assert len(entropy_encoder_block(b.astype(np.int64), 16)) == t
        from streamoptima_amd.bitstream import scan_order
        assert token_count(b.reshape(-1)[scan_order(16)], 16) == t
    assert entropy_encoder_block(g["tok_in16"][5].astype(np.int64), 16) == g["tok_list16_first"].tolist()


def test_synth_numpy_torch_identical():
    import torch
    from streamoptima_amd.synth import synth_sequence, synth_sequence_torch
    a = synth_sequence(3, 48, 80, seed=77)
    b = synth_sequence_torch(3, 48, 80, seed=77, device="cpu").numpy()
    assert (a == b).all()
    assert a.dtype == np.uint8 and a.std() > 10


def test_numpy_port_matches_reference_outputs():
    """oracle/ref_numpy.py (the CPU baseline) reproduces the reference's P-frame tokens and
    reconstruction (VBS off, golden vector 3)."""
    from oracle.ref_numpy import inter_rows
    g = golden("cif_p_vbs0.npz")
    tok, rec = inter_rows(g["cur"].astype(np.float64), g["ref"], range(0, 3))
    assert (rec[:48] == g["recon"][:48]).all()
    assert tok == int(g["tokens"].reshape(18, 22)[:3].sum())


def test_unsupported_modes_raise():
    from streamoptima_amd.Encoder import Y_Video_codec
    z = np.zeros((1, 32, 32), np.uint8)
    with pytest.raises(NotImplementedError):
        Y_Video_codec(32, 32, 1, 16, 16, 4, 1, 1, 0.015, False, y_only_frame_arr=z)
    with pytest.raises(ValueError):      # NameError on `mvp` in the reference (Encoder.py:609)
        Y_Video_codec(32, 32, 1, 16, 16, 4, 1, 0, 0.015, True, y_only_frame_arr=z, fast_me=True, ParallelMode=2)
    with pytest.raises(NotImplementedError):
        Y_Video_codec(32, 32, 1, 16, 16, 4, 1, 0, 0.015, False, y_only_frame_arr=z, ParallelMode=3)


def test_me_mode_selection():
    """fast_me / FMEEnable / ParallelMode pick the C-ABI ME mode (include/streamoptima.h)."""
    from streamoptima_amd import _lib
    from streamoptima_amd.Encoder import Y_Video_codec
    z = np.zeros((1, 32, 32), np.uint8)
    mk = lambda **k: Y_Video_codec(32, 32, 1, 16, 16, 4, 1, 0, 0.015, False, y_only_frame_arr=z, **k)  # noqa: E731
    assert mk()._me_mode() == _lib.ME_FULL
    assert mk(fast_me=True)._me_mode() == _lib.ME_FAST
    assert mk(fast_me=True, ParallelMode=2)._me_mode() == _lib.ME_FAST_PAR
    assert mk(ParallelMode=2)._me_mode() == _lib.ME_FULL
    assert mk(FMEEnable=True).FMEEnable


def test_engine_refuses_cpu_device():
    from streamoptima_amd import _lib
    from streamoptima_amd.engine import Engine
    with pytest.raises(_lib.HipPathError):
        Engine(32, 32, 16, 16, False, None, "cpu")


@pytest.mark.parametrize("name,rc", [("gop_cif_vbs0", None), ("gop_cif_vbs1_rc1", 1), ("gop_small_rc2", 2),
                                     ("gop_fme_vbs1", None), ("gop_fast_vbs1", None)])
def test_bitstream_parsers_on_reference_lines(name, rc):
    """differential_decoder_frame / entropy_decoder_frame (decoder.py:589-664) read the
    reference's own text lines back into its symbols (split, MVs, QTC, per-row QPs)."""
    import gzip
    import json
    from conftest import GOLDEN, golden
    from streamoptima_amd import bitstream as B
    g = golden(name + ".npz")
    js = json.load(gzip.open(os.path.join(GOLDEN, name + "_bitstream.json.gz"), "rt"))
    w = g["frames"].shape[2]
    for i, (ml, rl) in enumerate(zip(js["mv_lines"], js["residual_lines"])):
        ft, mvs, qps = B.differential_decoder_frame(ml, rc, w / 16)
        res = B.entropy_decoder_frame(rl, 16)
        assert ft == g["frame_type"][i]
        if rc:
            assert qps == g[f"qp_per_row{i}"].tolist()
        for b, (m, r) in enumerate(zip(mvs, res)):
            assert m[0] == r[0] == g[f"split{i}"][b]
            q = (np.asarray(r[1]).reshape(-1) if m[0] == 0
                 else np.concatenate([np.asarray(x).reshape(-1) for x in r[1]]))
            assert (q == g[f"qtc{i}"][b]).all()
            mv = g[f"mv{i}"][b]
            got = [m[1]] if m[0] == 0 else m[1]
            for k, v in enumerate(got):
                assert tuple(np.atleast_1d(v)) == tuple(np.atleast_1d(mv[k])), (i, b, k)
        # and the writer reproduces the line from the parsed symbols
        assert B.entropy_encoder_frame(res, 16) == rl


def test_entropy_block_round_trip():
    from streamoptima_amd import bitstream as B
    rng = np.random.default_rng(3)
    for n in (16, 8):
        for _ in range(200):
            q = rng.integers(-3, 4, size=(n, n)) * (rng.random((n, n)) < rng.random())
            assert (np.array(B.entropy_decoder_block(B.entropy_encoder_block(q, n), n)) == q).all()


def test_oracle_qp_map_rule():
    """Two-pass / ROI QP map: delta from the block's share of its row's pass-1
    tokens, ROI offsets on top, clamped."""
    from oracle import oracle as O
    t = np.array([10, 10, 10, 10,   40, 5, 2, 1], np.int32)      # two rows of 4 blocks
    qm = O.qp_map(t, 4, 2, 4, None, None, 0, 12)
    assert qm[:4].tolist() == [4, 4, 4, 4]                      # flat row: no change
    # row 2: sum 48, mean 12: 40 -> >=2x (+1, <4x), 5 -> <1/2 (-1), 2 -> <1/4 (-2), 1 -> -2
    assert qm[4:].tolist() == [5, 3, 2, 2]
    roi = np.array([-3, 0, 0, 9, 0, 0, 0, 0], np.int32)
    qm = O.qp_map(t, 4, 2, 4, [6, 1], roi, 0, 12)
    assert qm.tolist() == [3, 6, 6, 12, 2, 0, 0, 0]
    assert O.qp_map(None, 4, 2, 4, None, roi, 0, 12).tolist() == [1, 4, 4, 12, 4, 4, 4, 4]


def test_roi_rectangles_to_blocks():
    from streamoptima_amd.Encoder import Y_Video_codec
    z = np.zeros((1, 48, 64), np.uint8)
    enc = Y_Video_codec(48, 64, 1, 16, 16, 4, 1, 0, 0.015, False, y_only_frame_arr=z,
                        roi=[(0, 0, 32, 16, -2), (16, 16, 64, 48, 1)])
    assert enc.roi_block_offsets().reshape(3, 4).tolist() == [[-2, -2, 0, 0], [0, 1, 1, 1], [0, 1, 1, 1]]
    enc2 = Y_Video_codec(48, 64, 1, 16, 16, 4, 1, 0, 0.015, False, y_only_frame_arr=z,
                         roi=np.arange(12).reshape(3, 4))
    assert enc2.roi_block_offsets().tolist() == list(range(12))


def test_device_dct_header_bitwise_vs_oracle(tmp_path):
    """streamoptima_amd/csrc/so_dct.h (the kernels' FP64 DCT-II/III, with its exact
    power-of-two folds) compiled for the host matches the oracle's pocketfft restatement
    bit for bit on random, tie-heavy and dequantised vectors (tests/host/dct_host_check.cpp)."""
    import shutil
    import subprocess
    from oracle import oracle as O
    O.build()
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "dct_check")
    libdir = os.path.dirname(O.LIB_PATH)
    subprocess.run([gxx, "-O2", "-ffp-contract=off", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                    os.path.join(root, "tests", "host", "dct_host_check.cpp"), f"-L{libdir}", "-lso_oracle",
                    f"-Wl,-rpath,{libdir}", "-o", exe], check=True, capture_output=True)
    r = subprocess.run([exe, "300000"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
