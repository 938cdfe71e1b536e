"""GPU parity at the BENCHMARKED workloads: every frame of the 4K x 30 (configs[2]),
1080p -> 1088 x 30 (configs[1]), 4K x 120 seed 1 (configs[3]) and 4K ROI + two-pass RC
seed 2 (configs[4]) GOPs, and of their variants at the same sizes (VBS-on 4K and 1080p,
1080p FME / fast_me ParallelMode 0 and 2, 4K on low-texture and noise-only content),
bit-exact against the C oracle's per-frame digests
(tests/golden/large_gops.json, tests/golden/make_large_fixtures.py; the oracle itself is
pinned to the reference's 2-frame 1088p / 4K hashes by tests/test_oracle_golden.py)."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

from streamoptima_amd import _lib

pytestmark = pytest.mark.gpu

FIX = json.load(open(os.path.join(GOLDEN, "large_gops.json")))


def _codec(name, dev, **over):
    from streamoptima_amd.Encoder import Y_Video_codec
    from streamoptima_amd.workloads import ME_KW, RC_TABLES, WORKLOADS
    cfg = dict(WORKLOADS[name], **over)
    kw = dict(ME_KW[cfg.get("me", "full")])
    if cfg.get("rc"):
        kw.update(RCFlag=cfg["rc"], targetBR=cfg["target"], qp_rate_tables=RC_TABLES, roi=cfg.get("roi"))
    return cfg, Y_Video_codec(cfg["h"], cfg["w"], cfg["frames"], 16, 16, cfg["qp"], cfg["intra_dur"], 0, 0.015,
                              bool(cfg.get("vbs")), device=dev, **kw)


def _frames(cfg, dev):
    from streamoptima_amd.engine import alloc_planes
    from streamoptima_amd.synth import synth_sequence_torch
    from streamoptima_amd.workloads import padded
    h, w, f = cfg["h"], cfg["w"], cfg["frames"]
    fr = alloc_planes(f, padded(h), padded(w), dev, fill=128)
    fr[:, :h, :w].copy_(synth_sequence_torch(f, h, w, seed=cfg["seed"], device=dev,
                                             content=cfg.get("content", "bench")))
    return fr


def _check(name, syms, psnr=None):
    from streamoptima_amd.digest import symbols_digest
    fx = FIX[name]
    assert [s.frame_type for s in syms] == fx["frame_type"]
    bad = [i for i, s in enumerate(syms) if symbols_digest(s) != fx["frame_sha256"][i]]
    assert not bad, f"{name}: frames {bad[:10]} differ from the oracle"
    if psnr is not None:
        np.testing.assert_allclose(psnr, fx["psnr"], rtol=0, atol=1e-9)


@pytest.mark.parametrize("name", ["4k", "1080p", "4k120", "4k_rc2pass", "4k_vbs", "1080p_vbs", "1080p_fme",
                                  "1080p_fast", "1080p_fastpar", "4k_lowtex", "4k_noise"])
def test_benchmarked_gop_bit_exact(gpu, name):
    cfg, codec = _codec(name, gpu)
    frames = _frames(cfg, gpu)
    res = codec.encode_device(frames, cfg["intra_dur"])      # check=True: raises on a p_run timeout
    torch.cuda.synchronize()
    hp = frames.shape[1]
    sse = res["sse"].cpu().numpy()
    psnr = [10 * np.log10(255 ** 2 / (float(s) / (hp * cfg["w"]))) for s in sse]
    _check(name, res["symbols"], psnr)


@pytest.mark.parametrize("name", ["4k_lowtex", "4k", "1080p"])
def test_zero_skip_kernel_bit_exact_and_selected_by_content(gpu, name):
    """The plain run's zero-skip instantiation (SO_OPT_RUN_ZERO_SKIP: a wave whose blocks all
    quantised to zero skips the IDCT) gives the oracle's digests on flat and on textured content
    (forced on), and Engine.check_run selects it from the last run's share of all-zero blocks:
    on for the low-texture GOP, off for the textured ones."""
    cfg, codec = _codec(name, gpu)
    frames = _frames(cfg, gpu)
    eng = codec.engine()
    codec.encode_device(frames, cfg["intra_dur"])            # check=True: the content decision
    assert eng.zero_skip == (name == "4k_lowtex")
    eng.zero_skip = True
    res = codec.encode_device(frames, cfg["intra_dur"], check=False)
    torch.cuda.synchronize()
    eng.check_run()
    hp = frames.shape[1]
    sse = res["sse"].cpu().numpy()
    psnr = [10 * np.log10(255 ** 2 / (float(s) / (hp * cfg["w"]))) for s in sse]
    _check(name, res["symbols"], psnr)


def test_interleaved_gops_bit_exact(gpu):
    """encode_gops_device: two copies of the 1080p GOP (configs[1]) and a third GOP of the
    same frames reversed, their P-runs interleaved in ONE persistent launch: each copy equals
    the oracle's digests frame by frame, the reversed GOP equals its own encode_device."""
    from streamoptima_amd.digest import symbols_digest
    cfg, codec = _codec("1080p", gpu)
    from streamoptima_amd.engine import alloc_planes
    a = _frames(cfg, gpu)
    b = alloc_planes(*a.shape, gpu)
    b.copy_(a)
    c = alloc_planes(*a.shape, gpu)
    c.copy_(a.flip(0))
    ref_c = [symbols_digest(s) for s in codec.encode_device(c, cfg["intra_dur"])["symbols"]]
    res = codec.encode_gops_device([a, c, b], cfg["intra_dur"])
    torch.cuda.synchronize()
    hp = a.shape[1]
    for r in (res[0], res[2]):
        sse = r["sse"].cpu().numpy()
        _check("1080p", r["symbols"], [10 * np.log10(255 ** 2 / (float(s) / (hp * cfg["w"]))) for s in sse])
    assert [symbols_digest(s) for s in res[1]["symbols"]] == ref_c


def test_interleaved_gops_ragged_runs(gpu, monkeypatch):
    """Runs of different lengths and several I-frames per GOP (intra_dur 4 over 10 and 7
    frames: runs of 3, 3, 1 and 3, 2), more frames than one launch holds in total (chunked
    launches), on a frame with fewer tiles than the GPU's slots: equal to the per-frame
    kernels (SO_PIPELINE=0), both through encode_gops_device and through encode_device
    (which interleaves a GOP's own runs between I-frames)."""
    from streamoptima_amd.Encoder import Y_Video_codec
    from streamoptima_amd.digest import symbols_digest
    from streamoptima_amd.engine import alloc_planes
    from streamoptima_amd.synth import synth_sequence_torch
    h, w = 96, 256
    codec = Y_Video_codec(h, w, 10, 16, 16, 4, 4, 0, 0.015, False, device=gpu)

    def gop(n, seed):
        g = alloc_planes(n, h, w, gpu)
        g.copy_(synth_sequence_torch(n, h, w, seed=seed, device=gpu))
        return g
    gops = [gop(10, 3), gop(7, 4)] + [gop(12, 5 + k) for k in range(3)]
    monkeypatch.setenv("SO_PIPELINE", "0")
    exp = [[symbols_digest(s) for s in codec.encode_device(g, 4)["symbols"]] for g in gops]
    monkeypatch.delenv("SO_PIPELINE")
    res = codec.encode_gops_device(gops, 4)
    torch.cuda.synchronize()
    for g, r in enumerate(res):
        assert [symbols_digest(s) for s in r["symbols"]] == exp[g], g
        assert r["frame_type"] == [0 if i % 4 == 0 else 1 for i in range(gops[g].shape[0])]
    assert [symbols_digest(s) for s in codec.encode_device(gops[0], 4)["symbols"]] == exp[0]


@pytest.mark.parametrize("fused", ["0", "1"])
@pytest.mark.parametrize("roi", [None, [(100, 40, 400, 200, -2), (0, 150, 260, 272, 3)]])
def test_two_pass_run_matches_per_frame(gpu, monkeypatch, roi, fused):
    """so_encode_p_run_2pass -- the library-enqueued per-frame sequence (default) and both
    passes of every P-frame in one persistent launch (SO_OPT_RUN_2PASS_FUSED) -- against the
    Python-driven per-frame sequence pass 1 -> so_qp_map -> pass 2 (SO_PIPELINE=0), frame by
    frame including the QP maps, on a 640x272 GOP (5 x 9 tiles: pass-2 tasks of the 5-tile rows
    waiting on their row's pass 1), with and without ROI, two runs (intra_dur 5 of 11)."""
    from streamoptima_amd.Encoder import Y_Video_codec
    from streamoptima_amd.digest import symbols_digest
    from streamoptima_amd.engine import alloc_planes
    from streamoptima_amd.synth import synth_sequence_torch
    from streamoptima_amd.workloads import RC_TABLES
    h, w, f = 272, 640, 11
    codec = Y_Video_codec(h, w, f, 16, 16, 4, 5, 0, 0.015, False, RCFlag=3, targetBR="2 mbps",
                          qp_rate_tables=RC_TABLES, roi=roi, device=gpu)
    fr = alloc_planes(f, h, w, gpu)
    fr.copy_(synth_sequence_torch(f, h, w, seed=7, device=gpu))
    monkeypatch.setenv("SO_PIPELINE", "0")
    exp = codec.encode_device(fr, 5)
    exp_d = [symbols_digest(s) for s in exp["symbols"]]
    monkeypatch.delenv("SO_PIPELINE")
    monkeypatch.setenv("SO_RUN_2PASS", "1")
    with _lib.option(_lib.OPT_RUN_2PASS_FUSED, int(fused)):
        got = codec.encode_device(fr, 5)
    torch.cuda.synchronize()
    assert all("qp_map" in s.extra for s in got["symbols"])
    assert [symbols_digest(s) for s in got["symbols"]] == exp_d
    assert torch.equal(got["sse"], exp["sse"])


@pytest.mark.parametrize("h", [96, 64])
def test_two_pass_run_edge_shapes(gpu, monkeypatch, h):
    """The default two-pass run at the edge of the merged schedule's coverage: 96 rows (three
    tile rows, the fewest it takes: 2 tiles_x < ntiles) runs both passes in one launch, 64 rows
    (two tile rows) falls back to the per-frame sequence -- both against the Python-driven
    per-frame loop, frame by frame with the QP maps."""
    from streamoptima_amd.Encoder import Y_Video_codec
    from streamoptima_amd.digest import symbols_digest
    from streamoptima_amd.engine import alloc_planes
    from streamoptima_amd.synth import synth_sequence_torch
    from streamoptima_amd.workloads import RC_TABLES
    w, f = 640, 7
    codec = Y_Video_codec(h, w, f, 16, 16, 4, f, 0, 0.015, False, RCFlag=3, targetBR="2 mbps",
                          qp_rate_tables=RC_TABLES, roi=[(100, 16, 400, 60, -2)], device=gpu)
    fr = alloc_planes(f, h, w, gpu)
    fr.copy_(synth_sequence_torch(f, h, w, seed=5, device=gpu))
    monkeypatch.setenv("SO_PIPELINE", "0")
    exp = [symbols_digest(s) for s in codec.encode_device(fr, f)["symbols"]]
    monkeypatch.delenv("SO_PIPELINE")
    assert _lib.load().so_get_option(_lib.OPT_RUN_2PASS_FUSED) == 1
    got = codec.encode_device(fr, f)
    torch.cuda.synchronize()
    assert [symbols_digest(s) for s in got["symbols"]] == exp


def test_two_pass_run_longer_than_one_launch(gpu, monkeypatch):
    """The merged two-pass schedule over more P-frames than one launch holds (kRunMax = 32): 39
    P-frames at 96 rows (three tile rows, the fewest the merged schedule takes) run as two
    chunked launches, each with its own lag2 tail, and must equal the Python-driven per-frame
    sequence frame by frame with the QP maps."""
    from streamoptima_amd.Encoder import Y_Video_codec
    from streamoptima_amd.digest import symbols_digest
    from streamoptima_amd.engine import alloc_planes
    from streamoptima_amd.synth import synth_sequence_torch
    from streamoptima_amd.workloads import RC_TABLES
    h, w, f = 96, 640, 40
    codec = Y_Video_codec(h, w, f, 16, 16, 4, f, 0, 0.015, False, RCFlag=3, targetBR="2 mbps",
                          qp_rate_tables=RC_TABLES, roi=[(100, 16, 400, 60, -2)], device=gpu)
    fr = alloc_planes(f, h, w, gpu)
    fr.copy_(synth_sequence_torch(f, h, w, seed=9, device=gpu))
    monkeypatch.setenv("SO_PIPELINE", "0")
    exp = codec.encode_device(fr, f)
    exp_d = [symbols_digest(s) for s in exp["symbols"]]
    monkeypatch.delenv("SO_PIPELINE")
    assert _lib.load().so_p_run_2pass_fused(h, w) == 1
    got = codec.encode_device(fr, f)
    torch.cuda.synchronize()
    codec.engine().check_run()
    assert [symbols_digest(s) for s in got["symbols"]] == exp_d
    assert torch.equal(got["sse"], exp["sse"])


@pytest.mark.parametrize("roi", [None, [(100, 40, 400, 200, -2)]])
def test_two_pass_gop_replayed_as_hip_graph(gpu, roi):
    """bench.py --graph: a ROI / two-pass GOP captured once as a HIP graph (no host->device
    copy inside the capture: ROI offsets and row-QP schedules are uploaded once per content,
    Engine.device_const_i32) and replayed into poisoned outputs equals the eager encode."""
    from streamoptima_amd.Encoder import Y_Video_codec
    from streamoptima_amd.digest import symbols_digest
    from streamoptima_amd.engine import alloc_planes
    from streamoptima_amd.synth import synth_sequence_torch
    from streamoptima_amd.workloads import RC_TABLES
    h, w, f = 272, 640, 6
    codec = Y_Video_codec(h, w, f, 16, 16, 4, f, 0, 0.015, False, RCFlag=3, targetBR="2 mbps",
                          qp_rate_tables=RC_TABLES, roi=roi, device=gpu)
    fr = alloc_planes(f, h, w, gpu)
    fr.copy_(synth_sequence_torch(f, h, w, seed=11, device=gpu))
    exp = codec.encode_device(fr, f)
    exp_d = [symbols_digest(s) for s in exp["symbols"]]
    exp_sse = exp["sse"].clone()
    eng = codec.engine()
    pre = [eng.new_symbols(0 if i == 0 else 1) for i in range(f)]
    codec.encode_device(fr, f, symbols=pre, check=False)     # warm-up: workspaces, constants
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream(gpu)
    cap.wait_stream(torch.cuda.current_stream(gpu))
    with torch.cuda.stream(cap):
        with torch.cuda.graph(g, stream=cap):
            got = codec.encode_device(fr, f, symbols=pre, check=False)
    torch.cuda.current_stream(gpu).wait_stream(cap)
    for s in pre:
        s.qtc.fill_(0x5A5A)
        s.recon.fill_(3)
        s.tokens.fill_(-1)
    g.replay()
    torch.cuda.synchronize()
    eng.check_run()
    assert [symbols_digest(s) for s in got["symbols"]] == exp_d
    assert torch.equal(got["sse"], exp_sse)


def test_1080p_drop_in_encode_pads_to_1088(gpu, tmp_path, monkeypatch):
    """The public encode() on 1920x1080 host frames: pad_hw's 128 rows (Encoder.py:140-155,
    :1833), the 1088-row encode, PSNR over the padded plane -- the bench's 1080p record."""
    from streamoptima_amd.synth import synth_sequence
    cfg, codec = _codec("1080p", gpu, frames=6, intra_dur=6)
    codec.y_only_f_arr = synth_sequence(6, 1080, 1920, seed=cfg["seed"])
    monkeypatch.chdir(tmp_path)
    psnr = codec.encode(block_size=16)
    fx = FIX["1080p"]
    from streamoptima_amd.digest import symbols_digest
    for i, s in enumerate(codec._symbols):
        assert symbols_digest(s) == fx["frame_sha256"][i], i
    np.testing.assert_allclose(psnr, fx["psnr"][:6], rtol=0, atol=1e-9)


def test_4k120_poisoned_outputs(gpu):
    """Outputs written into buffers pre-filled with garbage (no stale-result masking): the
    first 40 frames of configs[3] -- two persistent launches, the second's frames depending
    on the first's."""
    cfg, codec = _codec("4k120", gpu, frames=40, intra_dur=120)
    eng = codec.engine()
    frames = _frames(cfg, gpu)
    pre = [eng.new_symbols(0 if i == 0 else 1) for i in range(40)]
    for s in pre:
        for t in (s.recon, s.qtc, s.mv, s.split, s.tokens, s.mae_num):
            t.view(torch.uint8).fill_(0xA5)
    res = codec.encode_device(frames, 120, symbols=pre)
    torch.cuda.synchronize()
    from streamoptima_amd.digest import symbols_digest
    fx = FIX["4k120"]
    bad = [i for i, s in enumerate(res["symbols"]) if symbols_digest(s) != fx["frame_sha256"][i]]
    assert not bad, bad


@pytest.mark.parametrize("h,w,intra_dur,content", [(272, 640, 5, "bench"), (1088, 1920, 4, "bench"),
                                                   (272, 640, 9, "noise")])
def test_vbs_run_matches_per_frame(gpu, monkeypatch, h, w, intra_dur, content):
    """VBSEnable in the persistent run (p_run_kernel<8, 0, true>: the block + sub-block dense
    search on the tile's LDS window and tq16_vbs's RD split) against the per-frame kernels
    (SO_PIPELINE=0: me_wave_kernel<16, true> + inter_tq_kernel<16, true>), frame by frame, on
    frames with edge tiles (640 = 5 tiles, 272 rows: a half tile row), several I-frames, and
    through encode_gops_device (runs of two GOPs interleaved in one launch).  Noise content
    overflows the bounds, so its tiles run the whole-tile dense scan over the window copies
    staged in the scratch."""
    from streamoptima_amd.Encoder import Y_Video_codec
    from streamoptima_amd.digest import symbols_digest
    from streamoptima_amd.engine import alloc_planes
    from streamoptima_amd.synth import synth_sequence_torch
    f = 9
    codec = Y_Video_codec(h, w, f, 16, 16, 4, intra_dur, 0, 0.015, True, device=gpu)
    assert codec.engine().pipelined_ok(1)
    fa = alloc_planes(f, h, w, gpu)
    fa.copy_(synth_sequence_torch(f, h, w, seed=21, device=gpu, content=content))
    fb = alloc_planes(f, h, w, gpu)
    fb.copy_(fa.flip(0))
    monkeypatch.setenv("SO_PIPELINE", "0")
    exp = [[symbols_digest(s) for s in codec.encode_device(g, intra_dur)["symbols"]] for g in (fa, fb)]
    monkeypatch.delenv("SO_PIPELINE")
    got = codec.encode_device(fa, intra_dur)
    torch.cuda.synchronize()
    assert [symbols_digest(s) for s in got["symbols"]] == exp[0]
    if content == "bench":
        assert int(sum(int(s.split.sum()) for s in got["symbols"][1:])) > 0   # some blocks split
    res = codec.encode_gops_device([fa, fb], intra_dur)
    torch.cuda.synchronize()
    for g in range(2):
        assert [symbols_digest(s) for s in res[g]["symbols"]] == exp[g], g


@pytest.mark.parametrize("content", ["noise", "lowtex", "noise_then_bench"])
def test_dense_predicted_tiles_match_per_frame(gpu, monkeypatch, content):
    """Tiles whose 4x4-cell bounds overflowed in the previous frame (p_run_kernel's tile
    predictor) scan every block densely over the window copies staged in the scratch -- against
    the per-frame kernels (SO_PIPELINE=0: me_wave_kernel's dense search), frame by frame, with
    edge tiles (640 = 5 tiles, 272 rows).  noise_then_bench: a scene change at frame 9 to
    textured content, the tiles still predicted dense until the probe frame (every 16th,
    SO_DENSE_PROBE), over 20 frames."""
    from streamoptima_amd.Encoder import Y_Video_codec
    from streamoptima_amd.digest import symbols_digest
    from streamoptima_amd.engine import alloc_planes
    from streamoptima_amd.synth import synth_sequence_torch
    h, w = 272, 640
    f = 20 if content == "noise_then_bench" else 9
    codec = Y_Video_codec(h, w, f, 16, 16, 4, f, 0, 0.015, False, device=gpu)
    assert codec.engine().pipelined_ok(1)
    fr = alloc_planes(f, h, w, gpu)
    if content == "noise_then_bench":
        fr[:9].copy_(synth_sequence_torch(f, h, w, seed=23, device=gpu, content="noise")[:9])
        fr[9:].copy_(synth_sequence_torch(f, h, w, seed=23, device=gpu)[9:])
    else:
        fr.copy_(synth_sequence_torch(f, h, w, seed=23, device=gpu, content=content))
    monkeypatch.setenv("SO_PIPELINE", "0")
    exp = [symbols_digest(s) for s in codec.encode_device(fr, f)["symbols"]]
    monkeypatch.delenv("SO_PIPELINE")
    got = codec.encode_device(fr, f)
    torch.cuda.synchronize()
    assert [symbols_digest(s) for s in got["symbols"]] == exp


@pytest.mark.parametrize("vbs,fme", [(False, False), (True, False), (False, True), (True, True)])
def test_fast_me_chain_speculation_matches_serial_walk(gpu, monkeypatch, vbs, fme):
    """fast_me mode 0 (Encoder.py:719-742, the predictor chain of :462-585): the segmented
    speculative chain (one wavefront per 32-block segment, warm-up guess, in-order check and
    redo) against the one-wavefront serial walk (SO_OPT_FASTME_SERIAL), frame by frame, on
    1920x1088 with and without VBS / FME -- and with no warm-up and 8-block segments, where
    nearly every guess is wrong and the redo path carries the result."""
    from streamoptima_amd.Encoder import Y_Video_codec
    from streamoptima_amd.digest import symbols_digest
    from streamoptima_amd.engine import alloc_planes
    from streamoptima_amd.synth import synth_sequence_torch
    h, w, f = 1088, 1920, 3
    codec = Y_Video_codec(h, w, f, 16, 16, 4, f, 0, 0.015, vbs, fast_me=True, FMEEnable=fme, device=gpu)
    fr = alloc_planes(f, h, w, gpu)
    fr.copy_(synth_sequence_torch(f, h, w, seed=11, device=gpu))

    def run():
        return [symbols_digest(s) for s in codec.encode_device(fr, f)["symbols"]]
    with _lib.option(_lib.OPT_FASTME_SERIAL, 1):
        exp = run()
    assert run() == exp
    with _lib.option(_lib.OPT_FASTME_WARMUP, 0), _lib.option(_lib.OPT_FASTME_SEGMENT, 8):
        assert run() == exp
