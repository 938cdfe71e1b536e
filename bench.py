#!/usr/bin/env python
"""Benchmark: encoded Mpixels/s of the StreamOptima per-block encode path on MI355X.

Workload (BASELINE.json configs[2], the 4K single-GPU config; 1080p with --config 1080p):
a 30-frame GOP (1 I-frame + 29 P-frames), 16x16 blocks, full-search ME +-16, QP 4,
intra_mode 0, nRefFrames 1, VBS off (headline VBS off, --vbs for the
variant), synthetic frames (streamoptima_amd/synth.py) already resident in HBM.
One step = one whole GOP encode (ME, residual, DCT/Q/IDCT, tokens, reconstruction and
PSNR SSE per frame), exactly the work Y_Video_codec.encode() launches per GOP.

Multi-GPU (torchrun), two modes:
  --shard gop (default): one process per GPU, each rank encodes its own independent GOP
      (seed = rank).  GOPs are independent units, so there is no data-path collective:
      weak scaling.
  --shard stripe (configs[3] semantics): all ranks encode ONE GOP, each its own block-row
      stripe of every frame, with one in-place all_gather of the reconstruction per frame
      over RCCL/xGMI (streamoptima_amd/dist.py): strong scaling.
Timing: barrier + synchronize on both sides, max over ranks.

Prints ONE JSON line on rank 0 (driver contract), including:
  roofline     — the dominant kernel (ME) timed live with HIP events on its stream
  cpu_baseline — the faithful numpy port of the reference loops on a bounded sample
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
# v_sad_u8 issue limit: one wave64 instruction (64 lanes x 4 byte-|diffs|) per 4 cycles per
# SIMD, 1024 SIMDs, 2.4 GHz.  tools/ubench_sad.cpp measured 5.60e11 wave-instr/s on the box
# (4.39 cycles) = 1.434e14 |diffs|/s = 91% of this.
SAD_PEAK_OPS = 1024 * 2.4e9 / 4 * 64 * 4
SAD_MEASURED_OPS = 5.603e11 * 256
VALU_PEAK_INSTR_S = 1024 * 2.4e9 / 4   # wave64 VALU instructions per second, all SIMDs
METRIC = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "BASELINE.json")))["metric"]

CONFIGS = {
    "4k": dict(workload="4K 30-frame I+P GOP (configs[2])", h=2160, w=3840, frames=30, qp=4),
    "1080p": dict(workload="1080p 30-frame I+P GOP (configs[1], 1920x1088 internal)", h=1080, w=1920,
                  frames=30, qp=4),
    "4k120": dict(workload="4K 120-frame I+P GOP (configs[3])", h=2160, w=3840, frames=120, qp=4),
    # configs[4]: ROI + two-pass RC (RCFlag 3, build extension); a centred ROI rectangle at
    # -2 QP, 50 mbps against a QP-rate table scaled to 4K rows (rc_schedule.json table x 11)
    "4k_rc2pass": dict(workload="4K 30-frame ROI + two-pass RC GOP (configs[4])", h=2160, w=3840, frames=30, qp=4,
                       rc=3, target="50 mbps", roi=[(1280, 720, 2560, 1440, -2)]),
}
RC_TABLES = [[v * 11 for v in (9000, 6000, 4000, 2600, 1700, 1100, 700, 450, 300, 200)],
             [v * 11 for v in (7000, 4500, 3000, 2000, 1300, 850, 550, 350, 230, 150)]]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="4k")
    ap.add_argument("--frames", type=int, default=None)
    ap.add_argument("--vbs", action="store_true", help="VBSEnable=True (lambda 0.015)")
    ap.add_argument("--cpu-rows", type=int, default=4, help="block rows per frame type for the CPU sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--kernel-reps", type=int, default=20)
    ap.add_argument("--shard", choices=("gop", "stripe"), default="gop",
                    help="multi-GPU: independent GOP per rank (weak) or block-row stripes of one GOP (strong)")
    ap.add_argument("--me", choices=("full", "fme", "fast", "fastpar", "fast_fme"), default="full",
                    help="ME variant: full search (headline), FMEEnable, fast_me (serial chain), fast_me under "
                         "ParallelMode 2, fast_me + FMEEnable")
    ap.add_argument("--graph", action="store_true",
                    help="replay the GOP as one captured HIP graph (measured slower than host launches here)")
    ap.add_argument("--pcie", action="store_true",
                    help="also time the PCIe-inclusive path (pinned host frames in, symbols out)")
    return ap.parse_args()


def dist_setup(backend: str = "nccl"):
    """One process per GPU (torchrun env).  backend "nccl" is RCCL on ROCm; the CPU tests
    drive the same code with "gloo"."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    elif backend == "nccl":
        torch.cuda.set_device(0)
    return world, rank, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def me_kernel_name(vbs: bool, me: str = "full") -> str:
    if me != "full":
        f = "true" if "fme" in me else "false"
        s = "true" if vbs else "false"
        return {"fme": f"me_fme_kernel<{s}>"}.get(me, f"me_fastpred_kernel<{f}, {s}, 16>")
    if os.environ.get("SO_ME_IMPL") == "dense" or vbs:
        return "me_wave_kernel<16, %s>" % ("true" if vbs else "false")
    return "me_sea2_kernel"


def kernel_roofline(codec, frames_dev, symbols, reps: int, me_variant: str = "full") -> dict:
    """Average duration of the ME launch (the dominant kernel) and of the TQ launch for a
    P-frame, measured with HIP events recorded on the launch stream.  The launches replay
    the GOP's own P-frame work: launch k encodes frame i = 1 + k % (F-1) against the
    reconstruction of frame i-1 from the timed GOP (the reference ME really searches, whose
    content sets how much the successive-elimination bound prunes)."""
    from streamoptima_amd import _lib
    eng = codec.engine()
    lib = _lib.load()
    h, w, bs, sr = eng.h, eng.w, eng.bs, eng.sr
    nf = frames_dev.shape[0]
    pairs = [(frames_dev[i], _lib.ref_array([symbols[i - 1].recon])) for i in range(1, nf)]
    state = {"k": 0}
    best = torch.empty((eng.nb, 4), dtype=torch.int32, device=eng.device)
    sub = torch.empty((eng.nb, 4, 4), dtype=torch.int32, device=eng.device) if eng.vbs else None
    sym = eng.new_symbols(1)
    st = _lib.stream_handle(eng.device)

    ws = eng.fme_workspace(1) if eng.fme else None

    def me():
        cur, refs = pairs[state["k"] % len(pairs)]
        state["k"] += 1
        if me_variant == "full":
            _lib.check(lib.so_me_full_search(cur.data_ptr(), refs, 1, h, w, bs, sr, best.data_ptr(), _lib.ptr(sub),
                                             st), "me")
        else:   # ME variant incl. its phase-plane build (FME)
            _lib.check(lib.so_me_search_ex(cur.data_ptr(), refs, 1, h, w, bs, sr, eng.me_mode, int(eng.fme), 1,
                                           _lib.ptr(ws), best.data_ptr(), _lib.ptr(sub), st), "me_ex")

    def tq():
        cur, refs = pairs[state["k"] % len(pairs)]
        state["k"] += 1
        _lib.check(lib.so_inter_tq_recon(cur.data_ptr(), refs, 1, h, w, bs, best.data_ptr(), _lib.ptr(sub),
                                         4, None, int(eng.vbs), eng.lam, sym.split.data_ptr(), sym.mv.data_ptr(),
                                         sym.qtc.data_ptr(), sym.tokens.data_ptr(), sym.mae_num.data_ptr(),
                                         sym.recon.data_ptr(), sym.sse.data_ptr(), st), "tq")

    def me_dense():
        old = os.environ.get("SO_ME_IMPL")
        os.environ["SO_ME_IMPL"] = "dense"
        try:
            me()
        finally:
            if old is None:
                os.environ.pop("SO_ME_IMPL")
            else:
                os.environ["SO_ME_IMPL"] = old

    # the product path of a plain GOP: the P-frames as one persistent launch (p_run_kernel)
    run_ok = (me_variant == "full" and eng.pipelined_ok(1) and codec.nRefFrames == 1
              and os.environ.get("SO_PIPELINE", "1") != "0" and not getattr(codec, "_rc_on", lambda: False)())
    run_outs = [eng.new_symbols(1) for _ in range(nf - 1)] if run_ok else None

    def run():
        eng.encode_p_run([frames_dev[i] for i in range(1, nf)], symbols[0].recon, 4, run_outs)

    todo = (("me", me), ("tq", tq), ("me_dense", me_dense)) if me_variant == "full" else (("me", me), ("tq", tq))
    if run_ok:
        todo = (("run", run),) + todo
    out = {"me_dense": float("nan"), "run": None}
    for name, fn in todo:
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        n_rep = max(2, reps // 10) if name == "run" else reps
        for _ in range(n_rep):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[name] = e0.elapsed_time(e1) / n_rep / 1e3  # seconds per launch
    nb = eng.nb
    d = 2 * sr + 1
    # algorithmic work of one ME launch:
    #   bytes: current + reference plane (1 B/px each) + one 16-B MV record per block
    #   SAD ops: valid candidates x bs^2 |differences|
    nbx, nby = w // bs, h // bs
    xs = np.arange(nbx) * bs
    ys = np.arange(nby) * bs
    dx = np.arange(-sr, sr + 1)
    vx = ((xs[:, None] + dx[None, :] >= 0) & (xs[:, None] + dx[None, :] < w - bs)).sum(1)
    vy = ((ys[:, None] + dx[None, :] >= 0) & (ys[:, None] + dx[None, :] < h - bs)).sum(1)
    cands = int(vx.sum()) * int(vy.sum())
    me_bytes = 2 * h * w + 16 * nb
    tq_bytes = 5 * h * w + 8 * nb          # cur + pred + recon + QTC int16 + symbols
    # one P-frame of the fused kernel: cur + ref read, recon + QTC int16 written (5 B/px), and
    # per block split 1 + mv 12 x int16 + tokens, mae, sse int32 (37 B)
    frame_bytes = 5 * h * w + 37 * nb
    return {"me_s": out["me"], "tq_s": out["tq"], "me_dense_s": out["me_dense"], "me_bytes": me_bytes, "tq_bytes": tq_bytes,
            "sad_ops": cands * bs * bs, "cands": cands, "d": d, "run_s": out["run"], "run_frames": nf - 1,
            "run_bytes": (nf - 1) * frame_bytes, "frame_bytes": frame_bytes}


def cpu_baseline(cfg, rows: int) -> dict:
    """Faithful numpy port (oracle/ref_numpy.py) on `rows` block rows of one P-frame and one
    I-frame, extrapolated to the whole GOP (1 I + frames-1 P)."""
    from oracle.ref_numpy import inter_rows, intra_rows
    from streamoptima_amd.synth import synth_sequence
    h, w = cfg["h"], cfg["w"]
    hp = -(-h // 16) * 16
    band = rows * 16 + 32
    seq = synth_sequence(2, band, w, seed=0)
    cur = seq[1].astype(np.float64)
    ref = seq[0]
    t0 = time.perf_counter()
    inter_rows(cur, ref, range(1, 1 + rows), qp=cfg["qp"])
    tp = (time.perf_counter() - t0) / rows
    t0 = time.perf_counter()
    intra_rows(cur, range(1, 1 + rows), qp=cfg["qp"])
    ti = (time.perf_counter() - t0) / rows
    nrows = hp // 16
    f = cfg["frames"]
    t_gop = nrows * (ti + (f - 1) * tp)
    return {"value": round(f * h * w / t_gop / 1e6, 6), "unit": "Mpx/s", "cores": 1, "kind": "port",
            "sample": f"{rows} interior block rows of a P-frame and of an I-frame at {w}x{h} "
                      f"({rows * w // 16} blocks each), numpy port of Encoder.py loops, "
                      f"extrapolated to {nrows} rows x (1 I + {f - 1} P); "
                      f"P {tp * nrows:.1f} s/frame, I {ti * nrows:.2f} s/frame",
            "host": platform.processor() or platform.machine(), "os_cpu_count": os.cpu_count()}


def psnr_delta_vs_reference(dev) -> dict:
    """Encode the reference's own 4-frame CIF GOP fixture (tests/golden/gop_cif_vbs0.npz,
    produced by the reference encoder, tests/golden/make_golden.py) on this GPU and compare
    PSNR per frame and the reconstructions with the reference's."""
    from streamoptima_amd.Encoder import Y_Video_codec
    g = np.load(os.path.join(ROOT, "tests", "golden", "gop_cif_vbs0.npz"))
    frames = g["frames"]
    f, h, w = frames.shape
    codec = Y_Video_codec(h, w, f, 16, 16, 4, 4, 0, 0.015, False, y_only_frame_arr=frames, device=dev)
    res = codec.encode_device(codec._upload_padded(frames), 4)
    torch.cuda.synchronize()
    sse = res["sse"].cpu().numpy()
    psnr = [10 * np.log10(255 ** 2 / (float(s) / (h * w))) for s in sse]
    same = all(np.array_equal(s.recon.cpu().numpy(), g["recon"][i]) for i, s in enumerate(res["symbols"]))
    return {"psnr_delta_db_max": float(np.max(np.abs(np.array(psnr) - g["psnr"]))), "bit_exact_recon": bool(same),
            "fixture": "reference encoder, CIF 4-frame GOP QP4 (tests/golden/gop_cif_vbs0.npz)"}


def pcie_inclusive(codec, cfg, frames_dev, reps: int = 2) -> dict:
    """GOP time including the upload of pinned host source planes and the download of every
    frame's symbol arrays (split, mv, qtc, tokens): the rate a host-memory caller sees."""
    f = frames_dev.shape[0]
    host = frames_dev.cpu().pin_memory()
    eng = codec.engine()
    pre = [eng.new_symbols(0 if i % f == 0 else 1) for i in range(f)]
    outs = [{k: torch.empty(getattr(p, k).shape, dtype=getattr(p, k).dtype).pin_memory()
             for k in ("split", "mv", "qtc", "tokens")} for p in pre]
    best = None
    for _ in range(reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        frames_dev.copy_(host, non_blocking=True)
        res = codec.encode_device(frames_dev, f, symbols=pre)
        for s, o in zip(res["symbols"], outs):
            for k, t in o.items():
                t.copy_(getattr(s, k), non_blocking=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    return {"pcie_inclusive_mpx_s": round(f * cfg["h"] * cfg["w"] / best / 1e6, 2),
            "pcie_inclusive_ms_per_gop": round(best * 1e3, 3)}


def main():
    args = parse()
    world, rank, local = dist_setup()
    cfg = dict(CONFIGS[args.config])
    if args.frames:
        cfg["frames"] = args.frames
    from streamoptima_amd.Encoder import Y_Video_codec
    from streamoptima_amd.engine import alloc_planes
    from streamoptima_amd.synth import synth_sequence_torch
    dev = torch.device("cuda", local)
    h, w, f = cfg["h"], cfg["w"], cfg["frames"]
    hp = -(-h // 16) * 16
    me_kw = {"full": {}, "fme": dict(FMEEnable=True), "fast": dict(fast_me=True),
             "fastpar": dict(fast_me=True, ParallelMode=2), "fast_fme": dict(fast_me=True, FMEEnable=True)}[args.me]
    if cfg.get("rc"):
        # RCFlag 3 without intra_thresh: no P->I switch, so no host read per frame
        me_kw.update(RCFlag=cfg["rc"], targetBR=cfg["target"], qp_rate_tables=RC_TABLES, roi=cfg.get("roi"))
    codec = Y_Video_codec(h, w, f, 16, 16, cfg["qp"], f, 0, 0.015, args.vbs, y_only_frame_arr=None, device=dev,
                          **me_kw)
    eng = codec.engine()
    stripe = args.shard == "stripe"
    frames = alloc_planes(f, hp, w, dev, fill=128)
    frames[:, :h, :].copy_(synth_sequence_torch(f, h, w, seed=0 if stripe else rank, device=dev))
    pre = [eng.new_symbols(0 if i % f == 0 else 1) for i in range(f)]
    if stripe:
        from streamoptima_amd.dist import StripeGOPEncoder
        senc = StripeGOPEncoder(eng)

        def step():
            rc = cfg.get("rc")
            return senc.encode(frames, f, cfg["qp"], qp_sched=codec.row_qp_schedule(eng.nby) if rc else None,
                               rc_flag=rc, intra_thresh=None, roi=codec.roi_block_offsets())
    else:
        def step():
            return codec.encode_device(frames, f, symbols=pre)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # --graph: the GOP's launch sequence is captured once into a HIP graph and replayed (same
    # kernels, same work per step).  Off by default: host launches measured faster here.  The
    # stripe shard's RCCL all_gather stays on the host path.
    graph = args.graph and not stripe
    if graph:
        g = torch.cuda.CUDAGraph()
        cap = torch.cuda.Stream(dev)
        cap.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(cap):
            with torch.cuda.graph(g, stream=cap):
                res_g = step()
        torch.cuda.current_stream(dev).wait_stream(cap)
        g.replay()
        torch.cuda.synchronize()

        def step():  # noqa: F811
            g.replay()
            return res_g
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    elapsed = max_over_ranks(time.perf_counter() - t0, world)
    psnr_mean = None
    sse = res["sse"].cpu().numpy()
    psnr_mean = float(np.mean([10 * np.log10(255 ** 2 / (s / (hp * w))) for s in sse if s > 0]))

    rl = kernel_roofline(codec, frames, res["symbols"], args.kernel_reps, args.me) if rank == 0 else None
    delta = psnr_delta_vs_reference(dev) if rank == 0 else None
    pcie = pcie_inclusive(codec, cfg, frames) if rank == 0 and args.pcie and not stripe else None
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu = cpu_baseline(cfg, args.cpu_rows)
    if rank != 0:
        barrier(world)
        return
    ms_per_step = elapsed / args.steps * 1e3
    units = 1 if stripe else world          # GOPs encoded per step across the job
    mpx = units * args.steps * f * h * w / elapsed / 1e6
    me_gbs = rl["me_bytes"] / rl["me_s"] / 1e9
    traffic_doc = {}
    pmc = os.path.join(ROOT, "profiles", "pmc_me_traffic.json")
    if os.path.exists(pmc):
        try:
            traffic_doc = json.load(open(pmc)).get(args.config + ("_vbs" if args.vbs else ""), {}).get("kernels", {})
        except Exception:
            traffic_doc = {}

    def traffic_of(kernel):
        hit = traffic_doc.get("so::" + kernel)
        return round(hit["hbm_bytes"]) if hit else None

    def valu_issue_of(kernel, launch_s):
        # VALU issue roofline: SQ_INSTS_VALU per launch (PMC, profiles/pmc_me_traffic.json)
        # against one wave64 VALU instruction per 4 cycles per SIMD, 1024 SIMDs at 2.4 GHz
        hit = traffic_doc.get("so::" + kernel)
        if not hit or "sq_insts_valu" not in hit:
            return None
        peak = VALU_PEAK_INSTR_S
        achieved = hit["sq_insts_valu"] / launch_s
        return {"valu_instrs": round(hit["sq_insts_valu"]), "achieved_instr_s": achieved, "peak_instr_s": peak,
                "frac": round(achieved / peak, 4)}

    me_k = me_kernel_name(args.vbs, args.me)
    me_part = {"kernel": me_k, "launch_us": round(rl["me_s"] * 1e6, 2), "achieved_gbs": round(me_gbs, 2),
               "algorithmic_bytes": rl["me_bytes"], "traffic": traffic_of(me_k),
               # dense-equivalent |diff| rate: the exhaustive search's candidates x 256 per
               # launch time.  The SEA kernel prunes exactly, so it can exceed the
               # v_sad_u8 issue peak; dense_me is the unpruned kernel on the same frame.
               "valu_sad": {"dense_equivalent_ops": rl["sad_ops"] / rl["me_s"], "peak_ops": SAD_PEAK_OPS,
                            "frac": round(rl["sad_ops"] / rl["me_s"] / SAD_PEAK_OPS, 4),
                            "measured_peak_ops": SAD_MEASURED_OPS, "candidates": rl["cands"]},
               "dense_me": {"kernel": "me_wave_kernel<16, %s>" % ("true" if args.vbs else "false"),
                            "launch_us": round(rl["me_dense_s"] * 1e6, 2),
                            "valu_sad_frac": round(rl["sad_ops"] / rl["me_dense_s"] / SAD_PEAK_OPS, 4)}}
    tq_part = {"kernel": "inter_tq_kernel<16, %s, false>" % ("true" if args.vbs else "false"),
               "launch_us": round(rl["tq_s"] * 1e6, 2),
               "achieved_gbs": round(rl["tq_bytes"] / rl["tq_s"] / 1e9, 2)}
    if args.me != "full":
        # the SAD-op accounting is the integer full search's; the variants report time only
        me_part["valu_sad"] = None
        me_part["dense_me"] = None
    if rl["run_s"]:
        # the product path: the GOP's 29 P-frames as ONE persistent launch of the fused
        # search + transform kernel (so_encode_p_run), timed with HIP events on its stream
        run_k = "p_run_kernel<8>"
        run_gbs = rl["run_bytes"] / rl["run_s"] / 1e9
        n_launch = -(-rl["run_frames"] // 32)       # so_encode_p_run: <= 32 frames per launch
        roofline = {"bound": "hbm", "kernel": run_k, "achieved": round(run_gbs, 2), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(run_gbs / HBM_PEAK_GBS, 5), "traffic": traffic_of(run_k),
                    "algorithmic_bytes": round(rl["run_bytes"] / n_launch),
                    "launch_us": round(rl["run_s"] / n_launch * 1e6, 2),
                    "frames_per_launch": round(rl["run_frames"] / n_launch, 2),
                    "valu_issue": valu_issue_of(run_k, rl["run_s"] / n_launch),
                    "per_frame_us": round(rl["run_s"] / rl["run_frames"] * 1e6, 2),
                    "note": "the fused kernel is VALU-bound (SEA search + FP64 pocketfft-exact DCT), not HBM-bound: "
                            "valu_issue is its roofline; components = the same work as separate launches",
                    "components": {"me_search": me_part, "transform": tq_part}}
    else:
        roofline = {"bound": "hbm", "kernel": me_k, "achieved": round(me_gbs, 2), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(me_gbs / HBM_PEAK_GBS, 5), "traffic": traffic_of(me_k),
                    "algorithmic_bytes": rl["me_bytes"], "launch_us": round(rl["me_s"] * 1e6, 2),
                    "valu_sad": me_part["valu_sad"], "dense_me": me_part["dense_me"], "tq_kernel": tq_part}
    line = {
        "metric": METRIC,
        "value": round(mpx, 2), "unit": "Mpx/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3), "higher_is_better": True, "scaling": "strong" if stripe else "weak",
        "vs_baseline": None, "dtype": "u8", "data": "synthetic (splitmix64 texture, +2/+1 px/frame motion)",
        "config": {"workload": cfg["workload"], "width": w, "height": h, "frames": f, "block_size": 16,
                   "search_range": 16, "qp": cfg["qp"], "vbs": bool(args.vbs), "nRefFrames": 1, "me": args.me,
                   "transform": "fp64 pocketfft-exact DCT",
                   "parallelism": f"stripe x{world} (all_gather recon per frame)" if stripe else f"gop-per-rank x{world}",
                   "launch": "hip-graph (one GOP per replay)" if graph else "host launches"},
        "roofline": roofline,
        "cpu_baseline": cpu,
        "psnr_mean_db": round(psnr_mean, 4),
        "psnr_delta_vs_reference": delta,
    }
    if pcie:
        line.update(pcie)
    if cpu:
        line["gpu_over_cpu"] = round(mpx / cpu["value"], 1)
    print(json.dumps(line), flush=True)
    barrier(world)


if __name__ == "__main__":
    main()
