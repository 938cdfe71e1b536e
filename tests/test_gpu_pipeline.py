"""ONE GOP split into block-row stripes with the hand-off inside the persistent launch
(streamoptima_amd/pipeline.py, so_encode_p_run_stripe): the concatenated stripes must be
bit-identical to the one-GPU GOP, i.e. to the C oracle's digests of the benchmarked
workloads (tests/golden/large_gops.json).

On a one-GPU box the ranks share the GPU: in one process on separate streams (peers'
buffers as plain pointers), and as two processes whose buffers are mapped by IPC
(hipIpcGetMemHandle / hipIpcOpenMemHandle, the path the ranks of an 8-GPU node take over
xGMI).  Each rank's persistent grid is capped (half the machine for all of them) so that all
ranks are resident together and the I-frame kernels of a slower rank still find CUs, and
at most 3 ranks share the GPU in one process: a process has 4 hardware queues
(GPU_MAX_HW_QUEUES), and two ranks' streams on one queue would serialise the ranks' persistent
kernels (each waiting on the other's hand-off until the 50 ms timeout flags the run)."""
import json
import os
import socket

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

FIX = json.load(open(os.path.join(GOLDEN, "large_gops.json")))


def _frames(name, dev, nframes=None):
    from streamoptima_amd.engine import alloc_planes
    from streamoptima_amd.synth import synth_sequence_torch
    from streamoptima_amd.workloads import WORKLOADS, padded
    cfg = dict(WORKLOADS[name])
    if nframes:
        cfg["frames"] = nframes
    h, w, f = cfg["h"], cfg["w"], cfg["frames"]
    fr = alloc_planes(f, padded(h), padded(w), dev, fill=128)
    fr[:, :h, :w].copy_(synth_sequence_torch(f, h, w, seed=cfg["seed"], device=dev))
    return cfg, fr


def _digest_concat(ranks, syms_per_rank, nframes):
    from streamoptima_amd.digest import frame_digest
    out = []
    for i in range(nframes):
        parts = [s[i] for s in syms_per_rank]
        arr = {k: np.concatenate([getattr(p, k).cpu().numpy() for p in parts]) for k in
               ("split", "mv", "qtc", "tokens", "mae_num")}
        arr["recon"] = np.concatenate([r.stripe_recon(i).cpu().numpy() for r in ranks])
        out.append(frame_digest(parts[0].frame_type, arr))
    return out


_STREAMS = []


def _streams(dev):
    """Three streams created once per process, each on a hardware queue of its own, for the
    ranks that share this GPU in one process: a persistent grid of one rank waits on the
    other's flags, so two ranks on one queue (the second grid queued behind the first) time out.
    Plain streams share the runtime's pool of GPU_MAX_HW_QUEUES queues, each new stream taking
    the least-used one, so two consecutive streams can land on the same queue -- observed: a
    `-k` subset of the suite deterministically timed out its frame-pipeline test, which passes
    alone and in the full suite.  A stream created with a CU mask (all CUs here) gets a queue
    of its own (hipExtStreamCreateWithCUMask); wrapped for torch as an ExternalStream."""
    if not _STREAMS:
        import ctypes
        import os
        hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
        ncu = torch.cuda.get_device_properties(dev).multi_processor_count
        words = (ncu + 31) // 32
        mask = (ctypes.c_uint32 * words)(*([0xFFFFFFFF] * words))
        with torch.cuda.device(dev):
            for _ in range(3):
                h = ctypes.c_void_p()
                rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(words), mask)
                assert rc == 0, f"hipExtStreamCreateWithCUMask: {rc}"
                _STREAMS.append(torch.cuda.ExternalStream(h.value, device=dev))
    return _STREAMS


@pytest.mark.parametrize("name,world,nframes", [("1080p", 2, 30), ("4k", 3, 12), ("4k", 2, 30)])
def test_stripe_run_in_process_matches_one_gpu(gpu, name, world, nframes):
    from streamoptima_amd.engine import Engine
    from streamoptima_amd.pipeline import StripeRunRank
    cfg, fr = _frames(name, gpu, nframes)
    h, w = fr.shape[1:]
    engines = [Engine(h, w, 16, 16, False, 0.015, gpu) for _ in range(world)]
    streams = _streams(gpu)[:world]
    cap = 768 // (2 * world)     # half the machine for the persistent grids: the other ranks'
    ranks = [StripeRunRank(engines[r], world, r, nframes, stream=streams[r], max_wg=cap) for r in range(world)]
    torch.cuda.synchronize()
    for r in range(world):
        ranks[r].connect(ranks[r - 1].info() if r > 0 else None, ranks[r + 1].info() if r < world - 1 else None)
    for rep in range(2):     # twice: the second GOP runs on epoch 2 over the first GOP's planes and flags
        syms = []
        for r in range(world):
            with torch.cuda.stream(streams[r]):
                syms.append(ranks[r].encode(fr, cfg["intra_dur"], cfg["qp"]))
        torch.cuda.synchronize()
        for r in ranks:
            r.check()
        got = _digest_concat(ranks, syms, nframes)
        exp = FIX[name]["frame_sha256"][:nframes]
        bad = [i for i, (a, b) in enumerate(zip(got, exp)) if a != b]
        assert not bad, f"rep {rep}: frames {bad[:10]} differ from the one-GPU GOP"
    for r in ranks:
        r.close()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _ipc_worker(rank, world, port, name, nframes, outdir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from streamoptima_amd.engine import Engine
        from streamoptima_amd.pipeline import PipelinedStripeGOPEncoder
        dev = torch.device("cuda:0")
        cfg, fr = _frames(name, dev, nframes)
        eng = Engine(fr.shape[1], fr.shape[2], 16, 16, False, 0.015, dev)
        enc = PipelinedStripeGOPEncoder(eng, nframes, max_wg=768 // (2 * world))
        res = enc.encode(fr, cfg["intra_dur"], cfg["qp"])
        torch.cuda.synchronize()
        enc.check()
        from streamoptima_amd.digest import frame_digest
        digs = []
        for i, s in enumerate(res["symbols"]):
            g = enc.gather_symbols(s, i)
            digs.append(frame_digest(g["frame_type"], {k: (v.cpu().numpy() if torch.is_tensor(v) else v)
                                                        for k, v in g.items()}))
        if rank == 0:
            with open(os.path.join(outdir, "digests.json"), "w") as fh:
                json.dump({"digests": digs, "sse": res["sse"].cpu().tolist()}, fh)
        dist.barrier()
        enc.close()
    finally:
        dist.destroy_process_group()


def test_stripe_run_two_processes_ipc(gpu, tmp_path):
    """Two ranks as two processes (one GPU, buffers mapped by IPC), 1080p GOP head."""
    import torch.multiprocessing as mp
    n = 10
    mp.start_processes(_ipc_worker, args=(2, _free_port(), "1080p", n, str(tmp_path)), nprocs=2,
                       start_method="spawn")
    got = json.load(open(tmp_path / "digests.json"))
    assert got["digests"] == FIX["1080p"]["frame_sha256"][:n]
    hp, w = 1088, 1920
    psnr = [10 * np.log10(255 ** 2 / (s / (hp * w))) for s in got["sse"]]
    np.testing.assert_allclose(psnr, FIX["1080p"]["psnr"][:n], rtol=0, atol=1e-9)


def _rc_codec(dev, n, rc, thresh):
    from streamoptima_amd.Encoder import Y_Video_codec
    from streamoptima_amd.workloads import RC_TABLES, WORKLOADS
    cfg = WORKLOADS["4k_rc2pass"]
    return Y_Video_codec(cfg["h"], cfg["w"], n, 16, 16, cfg["qp"], n, 0, 0.015, False, RCFlag=rc,
                         targetBR=cfg["target"], qp_rate_tables=RC_TABLES, roi=cfg["roi"], intra_thresh=thresh,
                         device=dev)


def _rc_stripe_worker(rank, world, port, n, rc, thresh, outdir):
    """dist.StripeGOPEncoder on the HIP engine: RC / ROI / two-pass GOPs as block-row stripes
    with one RCCL-style all_gather (gloo here) per reconstruction."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from streamoptima_amd.digest import frame_digest
        from streamoptima_amd.dist import StripeGOPEncoder
        dev = torch.device("cuda:0")
        cfg, fr = _frames("4k_rc2pass", dev, n)
        codec = _rc_codec(dev, n, rc, thresh)
        eng = codec.engine()
        enc = StripeGOPEncoder(eng)
        res = enc.encode(fr, n, cfg["qp"], qp_sched=codec.row_qp_schedule(eng.nby), rc_flag=rc, intra_thresh=thresh,
                         roi=codec.roi_block_offsets())
        digs = []
        for s in res["symbols"]:
            g = enc.gather_symbols(s)
            digs.append(frame_digest(g["frame_type"], {k: (v.cpu().numpy() if torch.is_tensor(v) else v)
                                                        for k, v in g.items()}))
        if rank == 0:
            with open(os.path.join(outdir, "digests.json"), "w") as fh:
                json.dump({"digests": digs, "ftypes": res["frame_type"], "sse": res["sse"].cpu().tolist()}, fh)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_rc_roi_stripes_two_processes(gpu, tmp_path):
    """configs[4] across ranks (dist.StripeGOPEncoder with the HIP Engine, 2 processes on one
    GPU): the 4K ROI + two-pass RC GOP head equals the oracle digests (QP maps gathered across
    the stripes), and an RCFlag 2 GOP with ROI whose intra_thresh makes some P-frames switch to
    intra (the all_reduce of the residual size, Encoder.py:1851-1856) equals the one-GPU encode."""
    import torch.multiprocessing as mp
    from streamoptima_amd.digest import symbols_digest
    n = 6
    mp.start_processes(_rc_stripe_worker, args=(2, _free_port(), n, 3, None, str(tmp_path)), nprocs=2,
                       start_method="spawn")
    got = json.load(open(tmp_path / "digests.json"))
    assert got["digests"] == FIX["4k_rc2pass"]["frame_sha256"][:n]
    psnr = [10 * np.log10(255 ** 2 / (s / (2160 * 3840))) for s in got["sse"]]
    np.testing.assert_allclose(psnr, FIX["4k_rc2pass"]["psnr"][:n], rtol=0, atol=1e-9)
    # RCFlag 2: a threshold between the P-frames' residual sizes, so the switch fires for some
    _, fr = _frames("4k_rc2pass", gpu, n)
    probe = _rc_codec(gpu, n, 2, 10 ** 12).encode_device(fr, n)
    sizes = sorted(int(s.tokens.sum()) for s in probe["symbols"][1:])
    thresh = (sizes[0] + sizes[-1]) // 2 if sizes[0] < sizes[-1] else sizes[0] - 1
    exp = _rc_codec(gpu, n, 2, thresh).encode_device(fr, n)
    assert 0 in exp["frame_type"][1:], "the threshold should switch a P-frame to intra"
    exp_d = [symbols_digest(s) for s in exp["symbols"]]
    mp.start_processes(_rc_stripe_worker, args=(2, _free_port(), n, 2, thresh, str(tmp_path)), nprocs=2,
                       start_method="spawn")
    got = json.load(open(tmp_path / "digests.json"))
    assert got["ftypes"] == exp["frame_type"]
    assert got["digests"] == exp_d
    assert got["sse"] == exp["sse"].cpu().tolist()


# ---- frame pipeline (consecutive frames on consecutive ranks, so_encode_p_run_fpipe) -------------
def _fpipe_rc_kw(name, eng, nframes):
    """FramePipeRank.encode's RC keywords of a workload (configs[4]: the row-QP schedule, two-pass,
    the ROI offsets), from the drop-in codec's own settings."""
    from streamoptima_amd.workloads import WORKLOADS
    if not WORKLOADS[name].get("rc"):
        return {}
    codec = _rc_codec(eng.device, nframes, 3, None)
    return dict(qp_row=codec.row_qp_schedule(eng.nby), two_pass=True,
                roi_dev=eng.device_const_i32(codec.roi_block_offsets()), qp_clamp=tuple(codec.qp_clamp))


@pytest.mark.parametrize("name,world,nframes", [("4k", 2, 12), ("4k", 3, 13), ("1080p", 2, 30), ("4k_rc2pass", 2, 8),
                                                ("4k_rc2pass", 3, 10), ("4k_vbs", 2, 8), ("1080p_vbs", 3, 10)])
def test_frame_pipeline_in_process_matches_one_gpu(gpu, name, world, nframes):
    """Rank g encodes frames g, g+N, ...; each frame's reference arrives tile by tile from the
    previous rank.  Whole-frame symbols and local reconstructions of every frame must equal
    the one-GPU GOP (oracle digests), twice in a row (epoch 2 over epoch 1's planes).
    4k_rc2pass: configs[4] (ROI + two-pass RC) on the frame pipeline, QP maps included; *_vbs:
    VBSEnable (block + sub-block search and the RD split inside the launch)."""
    from streamoptima_amd.digest import symbols_digest
    from streamoptima_amd.engine import Engine
    from streamoptima_amd.pipeline import FramePipeRank
    cfg, fr = _frames(name, gpu, nframes)
    h, w = fr.shape[1:]
    engines = [Engine(h, w, 16, 16, bool(cfg.get("vbs")), 0.015, gpu) for _ in range(world)]
    streams = _streams(gpu)[:world]
    cap = 768 // (2 * world)
    ranks = [FramePipeRank(engines[r], world, r, nframes, stream=streams[r], max_wg=cap) for r in range(world)]
    torch.cuda.synchronize()
    for r in range(world):
        ranks[r].connect(ranks[(r + 1) % world].info(), ranks[(r - 1) % world].info())
    rc_kw = [_fpipe_rc_kw(name, engines[r], nframes) for r in range(world)]
    for r in range(world):   # every rank's buffers before any rank's persistent grid runs
        ranks[r].prepare(nframes, rc_kw[r].get("qp_row"), rc_kw[r].get("two_pass", False))
    torch.cuda.synchronize()
    for rep in range(2):
        syms = {}
        for r in range(world):
            with torch.cuda.stream(streams[r]):
                syms.update(ranks[r].encode(fr, nframes, cfg["qp"], **rc_kw[r]))
        torch.cuda.synchronize()
        for r in ranks:
            r.check()
        got = [symbols_digest(syms[k]) for k in range(nframes)]
        exp = FIX[name]["frame_sha256"][:nframes]
        bad = [i for i, (a, b) in enumerate(zip(got, exp)) if a != b]
        assert not bad, f"rep {rep}: frames {bad[:10]} differ from the one-GPU GOP"
    for r in ranks:
        r.close()


def test_frame_pipeline_back_to_back_gops(gpu):
    """GOPs enqueued back to back with no synchronisation between them (bench.py's timed
    loop, FramePipelineGOPEncoder.encode(reduce=False)): a rank starts GOP k+1 while the
    other rank still encodes GOP k, overwriting landing slots under the next epoch.  Every
    GOP must still match its one-GPU encode: A (the fixture), then B (A's frames in reverse,
    against Y_Video_codec.encode_device), then A again."""
    from streamoptima_amd.digest import symbols_digest
    from streamoptima_amd.Encoder import Y_Video_codec
    from streamoptima_amd.engine import Engine
    from streamoptima_amd.pipeline import FramePipeRank
    name, world, nframes = "1080p", 2, 10
    cfg, fa = _frames(name, gpu, nframes)
    fb = fa.flip(0).contiguous()
    h, w = fa.shape[1:]
    codec = Y_Video_codec(h, w, nframes, 16, 16, cfg["qp"], nframes, 0, 0.015, False, device=gpu)
    exp_b = [symbols_digest(s) for s in codec.encode_device(fb, nframes)["symbols"]]
    exp_a = FIX[name]["frame_sha256"][:nframes]
    engines = [Engine(h, w, 16, 16, False, 0.015, gpu) for _ in range(world)]
    streams = _streams(gpu)[:world]
    ranks = [FramePipeRank(engines[r], world, r, nframes, stream=streams[r], max_wg=768 // (2 * world))
             for r in range(world)]
    torch.cuda.synchronize()
    for r in range(world):
        ranks[r].connect(ranks[(r + 1) % world].info(), ranks[(r - 1) % world].info())
    # every rank's buffers and the copies kept below allocated before any rank's persistent grid runs
    fields = ("split", "mv", "qtc", "tokens", "mae_num", "recon")
    mine = [ranks[r].prepare(nframes)[0] for r in range(world)]
    bufs = [[{k: {f: torch.empty_like(getattr(s, f)) for f in fields} for k, s in mine[r].items()}
             for r in range(world)] for _ in range(3)]
    torch.cuda.synchronize()
    saved = []
    for g, fr in enumerate((fa, fb, fa)):
        syms = {}
        for r in range(world):
            with torch.cuda.stream(streams[r]):
                syms.update(ranks[r].encode(fr, nframes, cfg["qp"]))
                # keep this GOP's symbols: the next encode() reuses the rank's buffers
                saved_r = bufs[g][r]
                for k, d in saved_r.items():
                    for f in fields:
                        d[f].copy_(getattr(syms[k], f))
                saved.append(saved_r)
    torch.cuda.synchronize()
    for r in ranks:
        r.check()
    import types
    for g, exp in enumerate((exp_a, exp_b, exp_a)):
        merged = {}
        for d in saved[g * world:(g + 1) * world]:
            merged.update(d)
        got = [symbols_digest(types.SimpleNamespace(frame_type=0 if k == 0 else 1, extra=None, **merged[k]))
               for k in range(nframes)]
        bad = [i for i, (a, b) in enumerate(zip(got, exp)) if a != b]
        assert not bad, f"GOP {g}: frames {bad[:10]} differ from the one-GPU encode"
    for r in ranks:
        r.close()


def _fpipe_worker(rank, world, port, name, nframes, outdir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from streamoptima_amd.engine import Engine
        from streamoptima_amd.pipeline import FramePipelineGOPEncoder
        dev = torch.device("cuda:0")
        cfg, fr = _frames(name, dev, nframes)
        eng = Engine(fr.shape[1], fr.shape[2], 16, 16, False, 0.015, dev)
        enc = FramePipelineGOPEncoder(eng, nframes, max_wg=768 // (2 * world))
        res = enc.encode(fr, nframes, cfg["qp"])
        torch.cuda.synchronize()
        enc.check()
        digs = enc.digests(res["symbols"], nframes)
        if rank == 0:
            with open(os.path.join(outdir, "digests.json"), "w") as fh:
                json.dump({"digests": digs, "sse": res["sse"].cpu().tolist()}, fh)
        dist.barrier()
        enc.close()
    finally:
        dist.destroy_process_group()


def test_frame_pipeline_two_processes_ipc(gpu, tmp_path):
    """Two ranks as two processes (one GPU, landing planes mapped by IPC), 4K GOP head."""
    import torch.multiprocessing as mp
    n = 8
    mp.start_processes(_fpipe_worker, args=(2, _free_port(), "4k", n, str(tmp_path)), nprocs=2, start_method="spawn")
    got = json.load(open(tmp_path / "digests.json"))
    assert got["digests"] == FIX["4k"]["frame_sha256"][:n]
    psnr = [10 * np.log10(255 ** 2 / (s / (2160 * 3840))) for s in got["sse"]]
    np.testing.assert_allclose(psnr, FIX["4k"]["psnr"][:n], rtol=0, atol=1e-9)


def test_in_process_ranks_must_fit_one_gpu(gpu):
    """Ranks sharing ONE GPU in a process (as these tests run them) can only make progress if
    every rank's persistent launch is resident at once: a rank whose launch cannot become
    resident would leave its peers polling for its tasks until the wait bound
    (profiles/r03/fpipe2p_fullcap_w3.log: three uncapped-share two-pass ranks, 256 timeouts
    each).  One rank per GPU always fits (its grid is its device's resident capacity; DESIGN.md
    section 6).  So the library refuses an in-process rank whose claim overflows the device
    (a lone rank: all of it; ranks sharing it: 3/4 of it together, the margin the time-shared
    runs have always had), and accepts capped ranks within that."""
    from streamoptima_amd import _lib
    from streamoptima_amd.engine import Engine
    from streamoptima_amd.pipeline import FramePipeRank
    cap = _lib.load().so_p_run_resident_workgroups(0)
    assert cap >= 256
    engines = [Engine(272, 3840, 16, 16, False, 0.015, gpu) for _ in range(3)]
    a = FramePipeRank(engines[0], 3, 0, 6, max_wg=0)            # uncapped: the whole device
    with pytest.raises(ValueError, match="resident workgroups"):
        FramePipeRank(engines[1], 3, 1, 6, max_wg=cap // 3)
    a.close()
    ranks = [FramePipeRank(engines[r], 3, r, 6, max_wg=cap // 4) for r in range(3)]   # 3/4 of the device, shared
    with pytest.raises(ValueError, match="resident workgroups"):
        FramePipeRank(engines[0], 3, 0, 6, max_wg=1)
    for r in ranks:
        r.close()


def test_claim_capacity_fits_every_run_kind(gpu):
    """The capacity ranks size their claims by (so_p_run_resident_workgroups) is the smallest of
    every run kernel they may launch: the stripe, frame-pipeline and two-pass kernels carry extra
    hand-off code and may fit fewer workgroups per CU than the one-GPU run."""
    from streamoptima_amd import _lib
    lib = _lib.load()
    for vbs, modes in ((0, (0, 1, 2, 3, 4)), (1, (0, 2))):
        cap = lib.so_p_run_resident_workgroups(vbs)
        per = {m: lib.so_p_run_mode_resident_workgroups(m, vbs) for m in modes}
        assert cap > 0 and all(v > 0 for v in per.values()), (cap, per)
        assert cap == min(per.values()), (vbs, cap, per)
    assert lib.so_p_run_mode_resident_workgroups(1, 1) < 0      # no VBS stripe run
    assert lib.so_p_run_mode_resident_workgroups(7, 0) < 0


def test_frame_pipeline_late_rank_is_not_a_stale_read(gpu):
    """A hand-off that arrives after its waits escalated to atomic reads (1 ms of polling) is a
    late flag, not a stale one: rank 1's grid is launched 20 ms before rank 0's, so its first
    waits poll through the escalation point and then see the flags arrive.  check() must report
    neither a timeout nor a stale read (the detector counts a flag only when a load issued after
    the RMW still misses what the RMW found), and the GOP must equal the one-GPU
    encode."""
    import time
    from streamoptima_amd.digest import symbols_digest
    from streamoptima_amd.engine import Engine
    from streamoptima_amd.pipeline import FramePipeRank
    name, world, nframes = "1080p", 2, 6
    cfg, fr = _frames(name, gpu, nframes)
    h, w = fr.shape[1:]
    engines = [Engine(h, w, 16, 16, False, 0.015, gpu) for _ in range(world)]
    streams = _streams(gpu)[:world]
    ranks = [FramePipeRank(engines[r], world, r, nframes, stream=streams[r], max_wg=768 // (2 * world))
             for r in range(world)]
    torch.cuda.synchronize()
    for r in range(world):
        ranks[r].connect(ranks[(r + 1) % world].info(), ranks[(r - 1) % world].info())
    for r in range(world):
        ranks[r].prepare(nframes)
    torch.cuda.synchronize()
    syms = {}
    for r in (1, 0):
        with torch.cuda.stream(streams[r]):
            syms.update(ranks[r].encode(fr, nframes, cfg["qp"]))
        if r == 1:
            time.sleep(0.02)
    torch.cuda.synchronize()
    for r in ranks:
        r.check()                                   # raises on a timeout or a stale read
        assert r.wait_health.stale_reads == 0
    got = [symbols_digest(syms[k]) for k in range(nframes)]
    assert got == FIX[name]["frame_sha256"][:nframes]
    for r in ranks:
        r.close()
