#!/usr/bin/env python
"""Benchmark: encoded Mpixels/s of the StreamOptima per-block encode path on MI355X.

Workload (BASELINE.json configs[2], the 4K single-GPU config; 1080p with --config 1080p):
a 30-frame GOP (1 I-frame + 29 P-frames), 16x16 blocks, full-search ME +-16, QP 4,
intra_mode 0, nRefFrames 1, VBS off (headline VBS off, --vbs for the
variant), synthetic frames (streamoptima_amd/synth.py) already resident in HBM.
One step = one whole GOP encode (ME, residual, DCT/Q/IDCT, tokens, reconstruction and
PSNR SSE per frame), exactly the work Y_Video_codec.encode() launches per GOP.

Multi-GPU (torchrun): one process per GPU, each rank encodes its own independent GOP
(seed = rank) — GOPs are independent units, so there is no data-path collective and the
scaling is weak.  Timing: barrier + synchronize on both sides, max over ranks.

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
SAD_PEAK_OPS = 256 * 4 * 32 * 2.4e9 * 4   # CUs x SIMD32 lanes x 2.4 GHz x 4 |diffs| per v_sad_u8

CONFIGS = {
    "4k": dict(workload="4K 30-frame I+P GOP (configs[2])", h=2160, w=3840, frames=30, qp=4),
    "1080p": dict(workload="1080p 30-frame I+P GOP (configs[1], 1920x1088 internal)", h=1080, w=1920,
                  frames=30, qp=4),
}


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
    return ap.parse_args()


def dist_setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
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
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def kernel_roofline(codec, frames_dev, reps: int) -> dict:
    """Average duration of the ME launch (the dominant kernel) and of the TQ launch for a
    P-frame, measured with HIP events recorded on the launch stream."""
    from streamoptima_amd import _lib
    eng = codec.engine()
    lib = _lib.load()
    h, w, bs, sr = eng.h, eng.w, eng.bs, eng.sr
    cur, ref = frames_dev[1], frames_dev[0]
    refs = _lib.ref_array([ref])
    best = torch.empty((eng.nb, 4), dtype=torch.int32, device=eng.device)
    sub = torch.empty((eng.nb, 4, 4), dtype=torch.int32, device=eng.device) if eng.vbs else None
    sym = eng.new_symbols(1)
    st = _lib.stream_handle(eng.device)

    def me():
        _lib.check(lib.so_me_full_search(cur.data_ptr(), refs, 1, h, w, bs, sr, best.data_ptr(), _lib.ptr(sub), st),
                   "me")

    def tq():
        _lib.check(lib.so_inter_tq_recon(cur.data_ptr(), refs, 1, h, w, bs, best.data_ptr(), _lib.ptr(sub),
                                         4, None, int(eng.vbs), eng.lam, sym.split.data_ptr(), sym.mv.data_ptr(),
                                         sym.qtc.data_ptr(), sym.tokens.data_ptr(), sym.mae_num.data_ptr(),
                                         sym.recon.data_ptr(), sym.sse.data_ptr(), st), "tq")

    out = {}
    for name, fn in (("me", me), ("tq", tq)):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[name] = e0.elapsed_time(e1) / reps / 1e3  # seconds per launch
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
    return {"me_s": out["me"], "tq_s": out["tq"], "me_bytes": me_bytes, "tq_bytes": tq_bytes,
            "sad_ops": cands * bs * bs, "cands": cands, "d": d}


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
    codec = Y_Video_codec(h, w, f, 16, 16, cfg["qp"], f, 0, 0.015, args.vbs, y_only_frame_arr=None, device=dev)
    eng = codec.engine()
    frames = alloc_planes(f, hp, w, dev, fill=128)
    frames[:, :h, :].copy_(synth_sequence_torch(f, h, w, seed=rank, device=dev))
    pre = [eng.new_symbols(0 if i % f == 0 else 1) for i in range(f)]

    def step():
        return codec.encode_device(frames, f, symbols=pre)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
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

    rl = kernel_roofline(codec, frames, args.kernel_reps) if rank == 0 else None
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu = cpu_baseline(cfg, args.cpu_rows)
    if rank != 0:
        barrier(world)
        return
    ms_per_step = elapsed / args.steps * 1e3
    mpx = world * args.steps * f * h * w / elapsed / 1e6
    me_gbs = rl["me_bytes"] / rl["me_s"] / 1e9
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_me_traffic.json")
    if os.path.exists(pmc):
        try:
            traffic = json.load(open(pmc)).get(args.config + ("_vbs" if args.vbs else ""), None)
        except Exception:
            traffic = None
    line = {
        "metric": "encoded Mpixels/sec (4K 30-frame I+P GOP, full-search ME +-16, QP 4)"
        if args.config == "4k" else "encoded Mpixels/sec (1080p 30-frame I+P GOP, full-search ME +-16, QP 4)",
        "value": round(mpx, 2), "unit": "Mpx/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8", "data": "synthetic (splitmix64 texture, +2/+1 px/frame motion)",
        "config": {"workload": cfg["workload"], "width": w, "height": h, "frames": f, "block_size": 16,
                   "search_range": 16, "qp": cfg["qp"], "vbs": bool(args.vbs), "nRefFrames": 1,
                   "transform": "fp64 pocketfft-exact DCT", "parallelism": f"gop-per-rank x{world}"},
        "roofline": {"bound": "hbm", "kernel": "me_fast_kernel", "achieved": round(me_gbs, 2),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(me_gbs / HBM_PEAK_GBS, 5),
                     "traffic": traffic, "algorithmic_bytes": rl["me_bytes"],
                     "launch_us": round(rl["me_s"] * 1e6, 2),
                     "valu_sad": {"achieved_ops": rl["sad_ops"] / rl["me_s"], "peak_ops": SAD_PEAK_OPS,
                                  "frac": round(rl["sad_ops"] / rl["me_s"] / SAD_PEAK_OPS, 4),
                                  "candidates": rl["cands"]},
                     "tq_kernel": {"launch_us": round(rl["tq_s"] * 1e6, 2),
                                   "achieved_gbs": round(rl["tq_bytes"] / rl["tq_s"] / 1e9, 2)}},
        "cpu_baseline": cpu,
        "psnr_mean_db": round(psnr_mean, 4),
    }
    if cpu:
        line["gpu_over_cpu"] = round(mpx / cpu["value"], 1)
    print(json.dumps(line), flush=True)
    barrier(world)


if __name__ == "__main__":
    main()
