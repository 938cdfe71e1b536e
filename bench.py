#!/usr/bin/env python
"""Benchmark: encoded Mpixels/s of the StreamOptima per-block encode path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config NAME]

Workloads (streamoptima_amd/workloads.py, BASELINE.json configs; synthetic splitmix64 frames
already resident in HBM; bs 16, full-search ME +-16, QP 4, intra_mode 0, nRefFrames 1,
VBS off):
  N = 1 (default --config 4k): configs[2], one 4K 30-frame I+P GOP per step; the line also
        carries a `records.1080p` entry for configs[1] (1920x1080 padded to 1088 rows),
        measured the same way in the same run, and `records.<cfg>_x<k>gop` entries: k
        independent GOPs per step with their P-runs interleaved in one persistent launch
        (--gops-in-flight, default 2; a GOP stream's throughput, every GOP parity-checked).
  N > 1 (default --config 4k120): configs[3], ONE 4K 120-frame GOP per step, sharded over
        the N ranks (strong scaling): by default the frame pipeline (each rank encodes one
        frame of every block of N, each reference arriving tile by tile from a ring
        neighbour over xGMI, the ring direction alternating per block;
        streamoptima_amd/pipeline.py FramePipelineGOPEncoder), self-checked before timing,
        else block-row stripes (--shard stripe; dist.py / pipeline.py).  --shard gop is the
        opt-in weak-scaling mode (an independent GOP per rank).
One step = one GOP through Y_Video_codec.encode_device(): every frame's ME, residual,
DCT/Q/IDCT, token count, reconstruction and per-block SSE.  It is encode()'s GPU work minus
the closed-loop decoder re-run (Encoder.py:1873, whose output the reference discards) and
minus the host package/file output.

`--gpus N` without a torchrun environment re-launches this script under
torch.distributed.run with N ranks BEFORE anything touches the GPU, and every rank checks
that WORLD_SIZE == N.  Timing: W untimed steps, then K steps bracketed by barrier +
synchronize, max over ranks.

After timing (never inside it) the script verifies its own output: the last timed step's
symbols are digested per frame (streamoptima_amd/digest.py) and compared with the C
oracle's digests of the same workload (tests/golden/large_gops.json), then one more step
runs into poisoned output buffers and is compared again.  `parity` in the line reports it.

Prints ONE JSON line on rank 0 (driver contract), including:
  roofline      -- the dominant kernel (p_run_kernel, the persistent fused search +
                   transform launch) timed live with HIP events on its stream: the required
                   HBM fraction, plus the VALU busy fraction from PMC counters
                   (profiles/pmc_me_traffic.json) -- the limit that actually binds it
  cpu_baseline  -- the numpy port of the reference loops (oracle/ref_numpy.py, calibrated
                   against the reference: profiles/cpu_port_calibration.json) on a bounded
                   sample, serial and with a Pool of worker processes
  pcie_inclusive -- BASELINE.md §4's timed region: pinned host Y planes in, symbols out
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import socket
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
# v_sad_u8 issue limit measured on the box (tools/ubench_sad.cpp): 4.39 cycles per wave64
# instruction at 8 waves/SIMD = 5.60e11 wave-instr/s = 1.434e14 |diffs|/s
SAD_MEASURED_OPS = 5.603e11 * 256
SAD_NOMINAL_OPS = 1.57e14      # 256 CUs x 2.4 GHz x 64 lanes x 4 bytes
N_SIMD = 1024                  # 256 CUs x 4 SIMDs
POOL_CAP = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)   # the GPU box's CPU share per GPU job
METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--record-repeats", type=int, default=3,
                    help="the `records` entries (not the headline) report the median of this many timed K-step runs")
    ap.add_argument("--config", default=None,
                    help="workload (streamoptima_amd/workloads.py); default 4k at N=1, 4k120 at N>1")
    ap.add_argument("--frames", type=int, default=None, help="override the workload's frame count (no parity)")
    ap.add_argument("--vbs", action="store_true",
                    help="VBSEnable=True (lambda 0.015): the workload's VBS-on variant (workloads.py, own fixture)")
    ap.add_argument("--cpu-rows", type=int, default=8,
                    help="block rows per frame type for the serial CPU sample (BASELINE.md §3: 8), spread over the "
                         "frame's height, edges included")
    ap.add_argument("--cpu-pool-rows", type=int, default=16, help="block rows for the Pool CPU sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-records", action="store_true", help="skip the 1080p record at N=1")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--gops-in-flight", type=lambda v: [int(x) for x in v.split(",") if x], default=[2],
                    help="N=1 records of a GOP stream: k GOPs per step with interleaved P-runs (comma list; '' = none)")
    ap.add_argument("--no-pcie", action="store_true")
    ap.add_argument("--pcie-last", action="store_true", help="measure the section-4 region after the records (A/B)")
    ap.add_argument("--kernel-reps", type=int, default=20)
    ap.add_argument("--exchange", choices=("p2p", "allgather"), default="p2p",
                    help="stripe hand-off: inside the persistent launch over xGMI (p2p, self-checked against "
                         "allgather before timing) or an RCCL all_gather of every reconstruction (allgather)")
    ap.add_argument("--shard", choices=("fpipe", "stripe", "gop"), default=None,
                    help="N>1: ONE GOP (strong, configs[3]) as a frame pipeline over the ranks (fpipe; falls back to "
                         "stripes if its self-check fails) or as block-row stripes, or a GOP per rank (weak); "
                         "default: stripes at N=2, fpipe from N=3")
    ap.add_argument("--me", choices=("full", "fme", "fast", "fastpar", "fast_fme"), default="full",
                    help="ME variant: full search (headline), FMEEnable, fast_me (serial chain), fast_me under "
                         "ParallelMode 2, fast_me + FMEEnable; selects the workload's variant where workloads.py "
                         "has one (1080p: 10-frame GOPs with oracle fixtures)")
    ap.add_argument("--no-content-records", action="store_true",
                    help="skip the N=1 records on low-texture / noise-only content")
    ap.add_argument("--no-graph", dest="graph", action="store_false",
                    help="one GOP per step by host launches instead of the default replay of one captured HIP "
                         "graph per GOP (N = 1 and --shard gop): the same kernels without the host launch gaps, "
                         "within noise to 1 %% faster (profiles/r04/bench_graph_ab.log)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal on a one-GPU host: every rank on cuda:0, gloo collectives, each rank's persistent "
                         "grid capped to a 1/(2N) share of the GPU (numbers are not a scaling measurement)")
    ap.add_argument("--inject-failure", default=None, metavar="WHAT",
                    help="test mode: make the named secondary measurement (e.g. records.1080p, cpu_baseline; with "
                         "--cpu-plumbing any name) raise, to check that the headline line still prints and the exit "
                         "status is nonzero")
    ap.add_argument("--detail-out", default=os.path.join(ROOT, "gpurun_out", "bench_detail.json"),
                    help="write the uncompacted line (every note and per-field source) here; '' = nowhere")
    ap.add_argument("--cpu-plumbing", action="store_true",
                    help="test mode: gloo + a trivial CPU stand-in engine (no encode, no GPU) to exercise the "
                         "rank launch, sharding, timing and JSON line on a CPU-only host")
    return ap.parse_args(argv)


# ---- ranks -----------------------------------------------------------------------------------
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(args) -> int:
    """`--gpus N` outside torchrun: run this script under torch.distributed.run with N ranks
    (one process per GPU) and return its exit code.  Called before any GPU call."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC (RCCL across processes)
    return subprocess.call(cmd, env=env)


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


def sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


# ---- parity -----------------------------------------------------------------------------------
def load_fixture(name: str):
    p = os.path.join(ROOT, "tests", "golden", "large_gops.json")
    if not os.path.exists(p):
        return None
    return json.load(open(p)).get(name)


def frame_digests(frames_syms) -> list:
    """Per-frame digests of host symbol dicts or FrameSymbols."""
    from streamoptima_amd.digest import frame_digest, symbols_digest
    out = []
    for s in frames_syms:
        out.append(frame_digest(s["frame_type"], s) if isinstance(s, dict) else symbols_digest(s))
    return out


def compare_digests(got: list, fx: dict) -> dict:
    from streamoptima_amd.digest import gop_digest
    exp = fx["frame_sha256"]
    bad = [i for i, (a, b) in enumerate(zip(got, exp)) if a != b]
    ok = len(got) == len(exp) and not bad
    return {"bit_exact": ok, "frames": len(got), "mismatched_frames": bad[:8],
            "gop_sha256": gop_digest(got), "expected_gop_sha256": fx["gop_sha256"]}


def poison(syms):
    for s in syms:
        for t in (s.recon, s.qtc, s.mv, s.split, s.tokens, s.mae_num):
            t.view(torch.uint8).fill_(0xA5)


# ---- roofline ----------------------------------------------------------------------------------
ALG_BYTES_DEF = "SURVEY.md section 8(d) / BASELINE.md section 4: 5 B/px (cur 1, ref 1, recon 1, QTC int16 2) + 8 B/block"


def alg_frame_bytes(hp: int, w: int, bs: int = 16) -> int:
    """Algorithmic HBM bytes of one P-frame (ALG_BYTES_DEF): 41.73 MB at 4K, 10.51 MB at 1088p."""
    return 5 * hp * w + 8 * (hp // bs) * (w // bs)


def kernel_roofline(codec, frames_dev, symbols, reps: int, components: bool = True) -> dict:
    """Average duration of p_run_kernel (the product path of a GOP's P-frames: one
    persistent launch per <= 32 frames, so_encode_p_run) measured with HIP events recorded
    on its launch stream, replaying the GOP's own P-frames against the reconstructions of
    the timed GOP; plus the separate ME (me_sea2_kernel) and transform (inter_tq_kernel)
    launches of the same work, for the component split."""
    from streamoptima_amd import _lib
    eng = codec.engine()
    lib = _lib.load()
    h, w, bs, sr = eng.h, eng.w, eng.bs, eng.sr
    nf = frames_dev.shape[0]
    st = _lib.stream_handle(eng.device)
    stream = torch.cuda.current_stream(eng.device)
    pairs = [(frames_dev[i], _lib.ref_array([symbols[i - 1].recon])) for i in range(1, nf)]
    state = {"k": 0}
    best = torch.empty((eng.nb, 4), dtype=torch.int32, device=eng.device)
    sym = eng.new_symbols(1)

    def me():
        cur, refs = pairs[state["k"] % len(pairs)]
        state["k"] += 1
        _lib.check(lib.so_me_full_search(cur.data_ptr(), refs, 1, h, w, bs, sr, best.data_ptr(), None, st), "me")

    def tq():
        cur, refs = pairs[state["k"] % len(pairs)]
        state["k"] += 1
        _lib.check(lib.so_inter_tq_recon(cur.data_ptr(), refs, 1, h, w, bs, best.data_ptr(), None, 4, None, 0, eng.lam,
                                         sym.split.data_ptr(), sym.mv.data_ptr(), sym.qtc.data_ptr(),
                                         sym.tokens.data_ptr(), sym.mae_num.data_ptr(), sym.recon.data_ptr(),
                                         sym.sse.data_ptr(), st), "tq")

    run_outs = [eng.new_symbols(1) for _ in range(nf - 1)]

    def run():
        eng.encode_p_run([frames_dev[i] for i in range(1, nf)], symbols[0].recon, 4, run_outs)

    out = {}
    sad_ops = None
    for name, fn in (("run", run), ("me", me), ("tq", tq)):
        if name != "run" and not components:
            continue
        # warm up for >= 0.2 s of GPU work: after an idle stretch the clock needs that long to
        # return to its working value (a 3-call warm-up read 15x too slow after the parity pass)
        t_end = time.perf_counter() + 0.2
        while time.perf_counter() < t_end:
            fn()
            torch.cuda.synchronize()
        torch.cuda.synchronize()
        if name == "run":
            # each launch between its own pair of events on the launch stream; the median of
            # max(6, reps / 2) launches (one slow launch after the parity pass's idle stretch
            # set the mean of two)
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(max(6, reps // 2))]
            for a, b in evs:
                a.record(stream)
                fn()
                b.record(stream)
            torch.cuda.synchronize()
            out[name] = float(np.median([a.elapsed_time(b) for a, b in evs])) / 1e3
        else:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(reps):
                fn()
            e1.record(stream)
            torch.cuda.synchronize()
            out[name] = e0.elapsed_time(e1) / reps / 1e3  # seconds per call
        if name == "run":
            # the executed SAD operations of the same work: one more (untimed) replay with the
            # kernel-side count on (SO_OPT_COUNT_SAD_OPS, words 66..67; off in timed runs)
            eng.check_run()
            eng.take_sad_ops()
            with _lib.option(_lib.OPT_COUNT_SAD_OPS, 1):
                fn()
                torch.cuda.synchronize()
            sad_ops = eng.take_sad_ops()
    eng.check_run()
    nb = eng.nb
    # algorithmic work: SAD ops = valid candidates x bs^2
    nbx, nby = w // bs, h // bs
    xs, ys, d = np.arange(nbx) * bs, np.arange(nby) * bs, np.arange(-sr, sr + 1)
    vx = ((xs[:, None] + d[None, :] >= 0) & (xs[:, None] + d[None, :] < w - bs)).sum(1)
    vy = ((ys[:, None] + d[None, :] >= 0) & (ys[:, None] + d[None, :] < h - bs)).sum(1)
    cands = int(vx.sum()) * int(vy.sum())
    # one P-frame's algorithmic bytes as SURVEY.md section 8(d) / BASELINE.md section 4 define them:
    # cur + ref read, recon + QTC int16 written (5 B/px) + 8 B/block (MV, ref, split, tokens)
    frame_bytes = alg_frame_bytes(h, w)
    return {"me_s": out.get("me"), "tq_s": out.get("tq"), "run_s": out["run"], "run_frames": nf - 1,
            "frame_bytes": frame_bytes, "me_bytes": 2 * h * w + 16 * nb, "tq_bytes": 5 * h * w + 8 * nb,
            "sad_ops": cands * bs * bs, "cands": cands, "executed_sad_ops": sad_ops, "vbs": eng.vbs,
            "zero_skip": bool(getattr(eng, "zero_skip", False))}


def pmc_record(config: str, kernel: str):
    """The committed PMC summary of `kernel` (a name prefix) for workload `config`
    (profiles/pmc_me_traffic.json, written by tools/traffic_json.py from rocprofv3 --pmc runs)."""
    p = os.path.join(ROOT, "profiles", "pmc_me_traffic.json")
    if not os.path.exists(p):
        return {}
    try:
        ks = json.load(open(p)).get(config, {}).get("kernels", {})
    except (ValueError, OSError):
        return {}
    # exact name first; else a name from before the run kernel's later template arguments (the
    # test hooks, round 5; the uniform QP, round 6) when those were false
    for k, v in ks.items():
        if k.startswith(kernel):
            return v
    alt = kernel
    while alt.endswith(", false>"):
        alt = alt[:-len(", false>")] + ">"
        for k, v in ks.items():
            if k.startswith(alt):
                return v
    return {}


def roofline_of(rl: dict, config: str) -> dict:
    """The dominant kernel's roofline line (task contract): p_run_kernel, the persistent fused
    search + transform launch of the GOP's P-frames, timed live with HIP events; the HBM
    fraction of its algorithmic bytes, the VALU busy fraction and HBM traffic from the
    committed PMC counters of the same workload, and the SAD fraction of the searches'
    EXECUTED v_sad byte operations (kernel-side count, SO_P_RUN_SAD_OPS_WORD)."""
    # the VBS workloads carry no row-QP schedule: the uniform-QP instantiation (so_me.hip UQP)
    kname = ("so::p_run_kernel<8, 0, true, false, true, false>" if rl["vbs"] else
             ("so::p_run_kernel<8, 0, false, false, false, true>" if rl.get("zero_skip") else
              "so::p_run_kernel<8, 0, false, false, false, false>"))
    n_launch = -(-rl["run_frames"] // 32)       # so_encode_p_run: <= 32 frames per launch
    launch_s = rl["run_s"] / n_launch
    alg = rl["run_frames"] * rl["frame_bytes"] / n_launch
    gbs = alg / launch_s / 1e9
    pm = pmc_record(config, kname)
    traffic = round(pm["hbm_bytes"]) if pm.get("hbm_bytes") else None
    valu = None
    if pm.get("sq_active_inst_valu") and pm.get("grbm_gui_active"):
        # SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES count quad-cycles summed over waves and
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md): the VALU busy
        # fraction = 4 * active / (kernel cycles per XCD * 1024 SIMDs)
        cyc = pm["grbm_gui_active"] / 8
        valu = {"valu_busy_frac": round(4 * pm["sq_active_inst_valu"] / (cyc * N_SIMD), 4),
                "sq_insts_valu": round(pm.get("sq_insts_valu", 0)),
                "cycles_per_valu_instr": round(4 * pm["sq_active_inst_valu"] / pm["sq_insts_valu"], 2)
                if pm.get("sq_insts_valu") else None,
                "waves_per_simd": round(4 * pm["sq_wave_cycles"] / (cyc * N_SIMD), 2) if pm.get("sq_wave_cycles") else None,
                "kernel_cycles": round(cyc), "effective_clock_ghz": round(cyc / launch_s / 1e9, 3),
                "source": f"profiles/pmc_me_traffic.json [{config}] (rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES "
                          "GRBM_GUI_ACTIVE ..., tools/gpu_traffic.sh)"}
    ex = rl.get("executed_sad_ops")
    sad = {"executed_byte_ops_per_launch": round(ex / n_launch) if ex else None,
           "executed_frac_of_measured_peak": round(ex / rl["run_s"] / SAD_MEASURED_OPS, 4) if ex else None,
           "executed_frac_of_nominal_peak": round(ex / rl["run_s"] / SAD_NOMINAL_OPS, 4) if ex else None,
           "dense_equivalent_byte_ops_per_launch": round(rl["sad_ops"] * rl["run_frames"] / n_launch),
           "dense_equivalent_frac_of_nominal_peak": round(rl["sad_ops"] * rl["run_frames"] / rl["run_s"]
                                                          / SAD_NOMINAL_OPS, 4),
           "note": "executed = every v_sad_u8 / v_sad_hi_u8 lane instruction of the searches (byte sums, bounds, "
                   "survivor and dense SADs) x 4 bytes, counted in the kernel; peaks: 1.434e14 |diff|/s measured "
                   "(tools/ubench_sad.cpp), 1.57e14 nominal (BASELINE.md section 4). The dense-equivalent count is the "
                   "reference's full scan (Encoder.py:688-715, valid candidates x 256), which the exact SEA search "
                   "mostly skips, so its 'fraction' can exceed 1"}
    out = {"bound": "hbm", "kernel": kname, "achieved": round(gbs, 2), "peak": HBM_PEAK_GBS,
           "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 5), "traffic": traffic,
           "traffic_note": "HBM bytes per launch from separate FETCH_SIZE / WRITE_SIZE passes; FETCH_SIZE x 2, the "
                           "factor measured for 4-B and 16-B coalesced reads (tools/ubench_fetch.cpp)",
           "algorithmic_bytes": round(alg), "algorithmic_bytes_def": ALG_BYTES_DEF,
           "launch_us": round(launch_s * 1e6, 2),
           "frames_per_launch": round(rl["run_frames"] / n_launch, 2),
           "per_frame_us": round(rl["run_s"] / rl["run_frames"] * 1e6, 2),
           "binding_limit": "valu",
           "valu_profile": valu, "sad": sad,
           "note": "frac is the required HBM fraction (algorithmic bytes / launch time / 8 TB/s); the kernel is "
                   "bound by VALU issue (SEA search + FP64 pocketfft-exact DCT), whose measured busy fraction is "
                   "valu_profile.valu_busy_frac (committed PMC counters of the same workload, not this run)"}
    if rl.get("me_s") and rl.get("tq_s"):
        out["components"] = {
            "me_search": {"kernel": "me_sea2_kernel", "launch_us": round(rl["me_s"] * 1e6, 2),
                          "achieved_gbs": round(rl["me_bytes"] / rl["me_s"] / 1e9, 2), "candidates": rl["cands"]},
            "transform": {"kernel": "inter_tq_kernel<16, false, false>", "launch_us": round(rl["tq_s"] * 1e6, 2),
                          "achieved_gbs": round(rl["tq_bytes"] / rl["tq_s"] / 1e9, 2)}}
    return out


def rc_roofline(codec, frames_dev, symbols, reps: int, config: str) -> dict:
    """configs[4] (ROI + two-pass RC): its P-run as the timed GOP enqueues it
    (so_encode_p_run_2pass) -- by default both passes in one persistent launch
    (p_run_kernel<8, 3>: each task the pass 2 of one tile, then the pass 1 of another), with
    SO_OPT_RUN_2PASS_FUSED = 0 the per-frame sequence (p_tile_kernel<8, true> pass 1,
    inter_tq_kernel<16, false, false, true> pass 2) -- replayed here with HIP events on the launch
    stream from the timed GOP's I-frame.  The HBM fraction of a P-frame's algorithmic bytes (as
    the one-pass roofline) over that run's time; the VALU busy fraction of the run kernel (the
    sequence: of its pass-1 kernel) from the committed PMC counters."""
    from streamoptima_amd import _lib
    e0 = codec.engine()
    fused = _lib.load().so_p_run_2pass_fused(e0.h, e0.w) == 1   # the library's own choice
    eng = codec.engine()
    qp_sched = codec.row_qp_schedule(eng.nby)
    qdev = eng.qp_row_tensor(qp_sched)
    roi = codec.roi_block_offsets()
    roi_dev = eng.device_const_i32(roi) if roi is not None else None
    lo, hi = codec.qp_clamp
    nf = frames_dev.shape[0]
    qp = codec.const_init_Qp
    outs = [eng.new_symbols(1) for _ in range(nf - 1)]
    maps = [torch.empty(eng.nb, dtype=torch.int32, device=eng.device) for _ in range(nf - 1)]
    stream = torch.cuda.current_stream(eng.device)

    def seq():
        eng.encode_p_run_2pass([frames_dev[i] for i in range(1, nf)], symbols[0].recon, qp, outs, maps,
                               qp_row=qp_sched, qp_row_dev=qdev, roi_dev=roi_dev, qp_lo=lo, qp_hi=hi)
    t_end = time.perf_counter() + 0.2
    while time.perf_counter() < t_end:
        seq()
        torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(max(6, reps // 2))]
    for a, b in evs:              # each run between its own events; the median (kernel_roofline)
        a.record(stream)
        seq()
        b.record(stream)
    torch.cuda.synchronize()
    per_frame = float(np.median([a.elapsed_time(b) for a, b in evs])) / 1e3 / (nf - 1)
    eng.check_run()
    frame_bytes = alg_frame_bytes(eng.h, eng.w)
    gbs = frame_bytes / per_frame / 1e9
    kname = "so::p_run_kernel<8, 3, false, false, false, false>" if fused else "so::p_tile_kernel<8, true>"
    # one persistent launch per <= 32 P-frames (fused); the sequence launches per frame
    n_launch = -(-(nf - 1) // 32) if fused else nf - 1
    launch_frames = (nf - 1) / n_launch
    pm = pmc_record(config, kname)
    valu = None
    if pm.get("sq_active_inst_valu") and pm.get("grbm_gui_active"):
        cyc = pm["grbm_gui_active"] / 8
        valu = {"kernel": kname[4:] + ("" if fused else " (pass 1)"),
                "valu_busy_frac": round(4 * pm["sq_active_inst_valu"] / (cyc * N_SIMD), 4),
                "waves_per_simd": round(4 * pm["sq_wave_cycles"] / (cyc * N_SIMD), 2) if pm.get("sq_wave_cycles") else None,
                "source": f"profiles/pmc_me_traffic.json [{config}]"}
    kdesc = ("two-pass P-run in one persistent launch (so_encode_p_run_2pass): p_run_kernel<8, 3, false, false, false, false>"
             if fused else "two-pass P-frame sequence (so_encode_p_run_2pass): p_tile_kernel<8, true> (pass 1) + "
             "inter_tq_kernel<16, false, false, true> (pass 2: QP map + transforms)")
    return {"bound": "hbm", "kernel": kdesc,
            "achieved": round(gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 5),
            "traffic": round(pm["hbm_bytes"]) if (fused and pm.get("hbm_bytes")) else None,
            "algorithmic_bytes": round(frame_bytes * launch_frames),
            "launch_us": round(per_frame * launch_frames * 1e6, 2), "frames_per_launch": round(launch_frames, 2),
            "per_frame_us": round(per_frame * 1e6, 2),
            "binding_limit": "valu", "valu_profile": valu,
            "algorithmic_bytes_def": ALG_BYTES_DEF,
            "note": "algorithmic bytes of the launch's P-frames over the measured time per launch; pass 1 re-reads "
                    "the current and reference rows pass 2 reads again"}


def gop_roofline(cfg, step_s: float, gops: int = 1) -> dict:
    """Whole-step HBM fraction: every frame's algorithmic bytes (ALG_BYTES_DEF) over the measured
    step time, for records whose step is more than the one persistent run (GOP streams, two-pass)."""
    from streamoptima_amd.workloads import padded
    h, w = padded(cfg["h"]), cfg["w"]
    alg = gops * cfg["frames"] * alg_frame_bytes(h, w)
    gbs = alg / step_s / 1e9
    return {"bound": "hbm", "scope": "whole step (every kernel of the GOP)", "achieved": round(gbs, 2),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 5), "algorithmic_bytes": alg}


# ---- CPU baseline --------------------------------------------------------------------------------
def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def cpu_baseline(cfg, rows: int, pool_rows: int) -> dict:
    """The numpy port of the reference loops (oracle/ref_numpy.py) on `rows` block rows of one
    P-frame and one I-frame, spread evenly over the frame's height with the first and last
    rows included (8 rows per frame type; edge rows have fewer valid
    candidates), serially (the reference's ParallelMode 0), and on `pool_rows` P-frame rows
    over a process Pool (the ParallelMode-2 analogue), each extrapolated to the whole GOP
    (1 I + frames-1 P).  The frames are the workload's own (synth.py, padded to 16 rows)."""
    from oracle.ref_numpy import inter_rows, inter_rows_pool, intra_rows
    from streamoptima_amd.synth import synth_sequence
    h, w = cfg["h"], cfg["w"]
    hp = -(-h // 16) * 16
    nrows, f = hp // 16, cfg["frames"]
    seq = np.full((2, hp, w), 128, np.uint8)
    seq[:, :h] = synth_sequence(2, h, w, seed=cfg["seed"], content=cfg.get("content", "bench"))
    cur = seq[1].astype(np.float64)
    ref = seq[0]
    sample = sorted({int(round(r)) for r in np.linspace(0, nrows - 1, rows)})
    psample = sorted({int(round(r)) for r in np.linspace(0, nrows - 1, pool_rows)})
    t0 = time.perf_counter()
    inter_rows(cur, ref, sample, qp=cfg["qp"])
    tp = (time.perf_counter() - t0) / len(sample)
    t0 = time.perf_counter()
    intra_rows(cur, sample, qp=cfg["qp"])
    ti = (time.perf_counter() - t0) / len(sample)
    t_gop = nrows * (ti + (f - 1) * tp)
    # BASELINE.md section 3 asks for Pool(os.cpu_count()).  os.cpu_count() on the GPU box is the
    # whole host (256 threads), but one GPU's job is allotted 16 of them (the box's worker-pool
    # rule: OMP_NUM_THREADS / MAX_JOBS are set to 16 there, and a pool sized to the host
    # oversubscribes the job's share): the pool gets min(affinity, 16) workers and the line
    # states both numbers.
    try:
        procs = min(len(os.sched_getaffinity(0)), POOL_CAP)
    except AttributeError:
        procs = min(os.cpu_count() or 1, POOL_CAP)
    t0 = time.perf_counter()
    inter_rows_pool(cur, ref, psample, procs, qp=cfg["qp"])
    tpp = (time.perf_counter() - t0) / len(psample)
    t_gop_pool = nrows * (ti / procs + (f - 1) * tpp)   # intra rows are as parallel (row-level, mode 2)
    calib = None
    cp = os.path.join(ROOT, "profiles", "cpu_port_calibration.json")
    if os.path.exists(cp):
        c = json.load(open(cp))
        calib = {"port_over_reference_time": c["p_frame"]["port_over_reference_time"],
                 "tokens_equal": c["tokens_equal"], "host": c["host"], "source": "profiles/cpu_port_calibration.json"}
    return {"value": round(f * h * w / t_gop / 1e6, 6), "unit": "Mpx/s", "cores": 1, "kind": "port",
            "sample": f"{len(sample)} block rows {sample} of a P-frame and of an I-frame at {w}x{hp} "
                      f"({len(sample) * w // 16} blocks each), numpy port of Encoder.py loops (oracle/ref_numpy.py), "
                      f"extrapolated to {nrows} rows x (1 I + {f - 1} P); "
                      f"P {tp * nrows:.1f} s/frame, I {ti * nrows:.2f} s/frame",
            "pool": {"value": round(f * h * w / t_gop_pool / 1e6, 6), "unit": "Mpx/s", "cores": procs,
                     "cores_note": f"Pool({procs}), not Pool(os.cpu_count() = {os.cpu_count()}): the GPU box allots "
                                   f"{POOL_CAP} CPUs to one GPU's job",
                     "sample": f"{len(psample)} P-frame block rows (spread over the frame) over Pool({procs}), one row per task "
                               f"(ParallelMode-2 analogue); P {tpp * nrows:.2f} s/frame"},
            "host": cpu_model(), "os_cpu_count": os.cpu_count(), "calibration": calib}


# ---- PCIe-inclusive --------------------------------------------------------------------------------
def pcie_inclusive(codec, cfg, frames_dev, reps: int = 10) -> dict:
    """BASELINE.md §4's timed region: pinned host Y planes -> HBM, the GOP encode, and the
    symbols back to pinned host memory -- as the dense arrays (split, mv, qtc, tokens), and as
    the packed stream (so_pack_frames: varint MVs + RLE token lists, plus per-frame SSE)."""
    from streamoptima_amd.hostmem import pinned_empty
    f = frames_dev.shape[0]
    host = pinned_empty(tuple(frames_dev.shape))     # page-locked by registration (hostmem.py)
    host.copy_(frames_dev.cpu())
    eng = codec.engine()
    pre = [eng.new_symbols(0 if i % cfg["intra_dur"] == 0 else 1) for i in range(f)]
    outs = [{k: pinned_empty(tuple(getattr(p, k).shape), getattr(p, k).dtype)
             for k in ("split", "mv", "qtc", "tokens")} for p in pre]
    d2h = sum(t.numel() * t.element_size() for o in outs for t in o.values())

    def dense():
        res = codec.encode_device(frames_dev, cfg["intra_dur"], symbols=pre, check=False)
        for s, o in zip(res["symbols"], outs):
            for k, t in o.items():
                t.copy_(getattr(s, k), non_blocking=True)
        return None

    from streamoptima_amd.hoststream import HostStreamEncoder
    hs = HostStreamEncoder(codec, f, chunk=2)
    got = {}

    def packed_run():
        got.update(hs.encode(host, cfg["intra_dur"]))
        return sum(got["bytes"]) + 8 * f

    med, reps_ms = {}, {}

    def timed(fn):
        ts, nbytes = [], None
        for _ in range(reps + 2):      # the first two calls warm the path (allocations, first copies)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            nbytes = fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        med[fn.__name__] = float(np.median(ts[2:]))
        reps_ms[fn.__name__] = [round(t * 1e3, 3) for t in ts]
        return min(ts[2:]), nbytes

    def dense_timed():
        frames_dev.copy_(host, non_blocking=True)
        return dense()

    best, _ = timed(dense_timed)
    codec.engine().check_run()
    # the packed streams must be those of the (fixture-checked) resident encode's symbols
    offs, packed = eng.pack_symbols(pre)
    best_p, d2h_p = timed(packed_run)
    same = all(torch.equal(got["packed"][i], packed[i, :int(offs[i, -1])].cpu()) for i in range(f))
    px = f * cfg["h"] * cfg["w"]
    # the link's own rates on this box: the GOP's pinned Y planes up alone, and as many bytes down
    # alone (copy engines, no kernel) -- the peaks the region's PCIe roofline is measured against
    dn = pinned_empty((host.numel(),))
    flat = frames_dev.view(-1)[:host.numel()]

    def up_only():
        frames_dev.copy_(host, non_blocking=True)

    def down_only():
        dn.copy_(flat, non_blocking=True)

    def rate(fn):
        ts = []
        for _ in range(reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return host.numel() / min(ts[1:]) / 1e9
    h2d_gbs, d2h_gbs = rate(up_only), rate(down_only)
    link = {"h2d_gbs": round(h2d_gbs, 2), "d2h_gbs": round(d2h_gbs, 2), "bytes": int(host.numel()),
            "method": "one pinned copy of the GOP's planes each way alone (copy engine, no kernel), best of "
                      f"{reps} after one warm-up"}
    up_gbs = int(host.numel()) / best_p / 1e9
    down_gbs = int(d2h_p) / best_p / 1e9
    return {"region": "BASELINE.md §4 (pinned host Y planes in, symbols back in pinned host memory)",
            "mpx_s": round(px / best_p / 1e6, 2), "ms_per_gop": round(best_p * 1e3, 3),
            "ms_per_gop_median": round(med["packed_run"] * 1e3, 3), "reps": reps,
            "rep_ms": reps_ms.get("packed_run"),
            "h2d_bytes": int(host.numel()), "d2h_bytes": int(d2h_p), "packed_equals_resident_symbols": bool(same),
            "link": link,
            "roofline": {"bound": "pcie", "achieved": round(up_gbs, 2), "peak": link["h2d_gbs"], "unit": "GB/s",
                         "frac": round(up_gbs / h2d_gbs, 4), "direction": "h2d (the binding one: the raw Y planes)",
                         "d2h": {"achieved": round(down_gbs, 2), "peak": link["d2h_gbs"],
                                 "frac": round(down_gbs / d2h_gbs, 4)},
                         "note": "bytes moved in the region / its time, against the link's measured one-way rate; "
                                 "both directions run at once (full duplex)"},
            "note": "streamoptima_amd/hoststream.py: per-frame H2D on one copy stream, P-runs of 2 frames + "
                    "so_pack_frames on the compute stream, packed symbol stream + per-frame SSE D2H on a second "
                    "copy stream, all overlapped; the timed region of BASELINE.md §4",
            "dense": {"mpx_s": round(px / best / 1e6, 2), "ms_per_gop": round(best * 1e3, 3), "d2h_bytes": int(d2h),
                      "note": "serial: H2D, one encode, dense split / mv / int16 QTC / tokens arrays D2H"}}


# ---- one workload ---------------------------------------------------------------------------------
def build_codec(cfg, args, dev):
    from streamoptima_amd.Encoder import Y_Video_codec
    from streamoptima_amd.workloads import ME_KW, RC_TABLES
    me_kw = dict(ME_KW[cfg.get("me", "full")])
    if cfg.get("rc"):
        # RCFlag 3 without intra_thresh: no P->I switch, so no host read per frame
        me_kw.update(RCFlag=cfg["rc"], targetBR=cfg["target"], qp_rate_tables=RC_TABLES, roi=cfg.get("roi"))
    return Y_Video_codec(cfg["h"], cfg["w"], cfg["frames"], 16, 16, cfg["qp"], cfg["intra_dur"], 0, 0.015,
                         bool(cfg.get("vbs")), y_only_frame_arr=None, device=dev, **me_kw)


def make_frames(cfg, dev, seed):
    from streamoptima_amd.engine import alloc_planes
    from streamoptima_amd.synth import synth_sequence_torch
    from streamoptima_amd.workloads import padded
    h, w, f = cfg["h"], cfg["w"], cfg["frames"]
    frames = alloc_planes(f, padded(h), padded(w), dev, fill=128)     # pad_hw: 128 below row h
    frames[:, :h, :w].copy_(synth_sequence_torch(f, h, w, seed=seed, device=dev, content=cfg.get("content", "bench")))
    return frames


def time_steps(step, world, steps, warmup, dev):
    for _ in range(warmup):
        step()
    sync(dev)
    barrier(world)
    sync(dev)
    t0 = time.perf_counter()
    res = None
    for _ in range(steps):
        res = step()
    sync(dev)
    barrier(world)
    sync(dev)
    return max_over_ranks(time.perf_counter() - t0, world), res


def run_single(cfg, args, dev, parity: bool):
    """One GOP per step on this GPU (N = 1, or --shard gop at N > 1)."""
    codec = build_codec(cfg, args, dev)
    eng = codec.engine()
    frames = make_frames(cfg, dev, cfg["seed"])
    f = cfg["frames"]
    pre = [eng.new_symbols(0 if i % cfg["intra_dur"] == 0 else 1) for i in range(f)]

    def step():
        return codec.encode_device(frames, cfg["intra_dur"], symbols=pre, check=False)
    graph = args.graph
    # one eager GOP first, and its wait-health check: the check also picks the plain run's kernel
    # for this content (Engine.zero_skip: the all-zero-wave IDCT skip where most blocks quantise
    # to zero), which the captured graph then replays
    step()
    torch.cuda.synchronize()
    eng.check_run()
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
    return codec, frames, pre, step


def psnr_delta(sse, fx, hp: int, w: int) -> dict | None:
    """PSNR per frame from the timed output's SSE (calculate_metrics, Encoder.py:934-935, over
    the padded plane as encode() computes it, :1869) against the oracle fixture's PSNR list:
    the metric's "PSNR delta vs reference"."""
    if sse is None or fx is None or "psnr" not in fx:
        return None
    vals = sse.cpu().numpy() if torch.is_tensor(sse) else np.asarray(sse)
    got = [float("inf") if s == 0 else 10 * np.log10(255 ** 2 / (float(s) / (hp * w))) for s in vals]
    # both inf (an exact frame on both sides): equal; one inf and one finite: a mismatch (inf)
    d = [abs(a - b) if (np.isfinite(a) and np.isfinite(b)) else (0.0 if a == b else float("inf"))
         for a, b in zip(got, fx["psnr"])]
    return {"psnr_delta_db_max": float(max(d)) if d else None, "frames": len(got),
            "psnr_mean_db": round(float(np.mean([g for g in got if np.isfinite(g)])), 4),
            "tolerance_db": 1e-4}


def parity_of(res, name, cfg, redo=None, sse=None) -> dict | None:
    """Digests of the timed output vs the oracle fixture; `redo()` re-runs one step into
    poisoned buffers and returns its symbols; `sse` (per-frame, device or host) adds the PSNR
    delta against the fixture's PSNR list."""
    from streamoptima_amd.workloads import padded
    fx = load_fixture(name)
    if fx is None:
        return {"bit_exact": None, "note": f"no oracle fixture for workload {name!r}"}
    got = frame_digests(res)
    out = compare_digests(got, fx)
    pd = psnr_delta(sse, fx, padded(cfg["h"]), cfg["w"])
    if pd is not None:
        out["psnr_delta_db"] = pd["psnr_delta_db_max"]
    if redo is not None:
        again = compare_digests(frame_digests(redo()), fx)
        out["poisoned_rerun_bit_exact"] = again["bit_exact"]
    out["fixture"] = "tests/golden/large_gops.json (C oracle, tests/golden/make_large_fixtures.py)"
    return out


def time_steps_median(step, args, dev):
    """Median over --record-repeats timed K-step runs (warm-up once): one host or box stall
    in a run of a few milliseconds would otherwise set a secondary record.  Returns
    (elapsed of the median run, its last result, every run's ms per step)."""
    runs = []
    for r in range(max(1, args.record_repeats)):
        elapsed, res = time_steps(step, 1, args.steps, args.warmup if r == 0 else 0, dev)
        runs.append((elapsed, res))
    order = sorted(range(len(runs)), key=lambda i: runs[i][0])
    elapsed, res = runs[order[len(order) // 2]]
    return elapsed, res, [round(e / args.steps * 1e3, 3) for e, _ in runs]


def dense_fallback_of(eng, cfg, step) -> dict:
    """The fraction of one GOP's P-frame blocks whose exact SEA search took the dense path
    (one extra, untimed step; the persistent run's fallback word)."""
    eng.take_fallback_count()
    step()
    eng.check_run()
    p_blocks = (cfg["frames"] - -(-cfg["frames"] // cfg["intra_dur"])) * eng.nb
    fb = eng.take_fallback_count()
    return {"blocks": fb, "p_blocks": p_blocks, "frac": round(fb / p_blocks, 5),
            "note": "P-frame blocks searched dense: the 4x4-cell bound left more survivors than the list holds (384, "
                    "also for a VBS block and its sub-blocks), or the tile "
                    "searched dense from the start because the same tile of the previous frame mostly overflowed "
                    "(SO_P_RUN_FALLBACK_WORD, one GOP)"}


def record_single(name: str, args, dev) -> dict:
    """Another workload measured like the headline (one GOP per step, median of
    --record-repeats timed runs, parity-checked): configs[1] (1080p) and the content-dependence
    records (4k_lowtex, 4k_noise), which also report the fraction of P-frame blocks whose exact
    SEA search took the dense fallback."""
    from streamoptima_amd.workloads import WORKLOADS, padded
    cfg = dict(WORKLOADS[name])
    codec, frames, pre, step = run_single(cfg, args, dev, True)
    eng = codec.engine()
    elapsed, res, runs = time_steps_median(step, args, dev)
    eng.check_run()
    mpx = args.steps * cfg["frames"] * cfg["h"] * cfg["w"] / elapsed / 1e6
    rec = {"workload": cfg["workload"], "value": round(mpx, 2), "unit": "Mpx/s",
           "ms_per_step": round(elapsed / args.steps * 1e3, 3), "ms_per_step_runs": runs, "width": cfg["w"],
           "height": cfg["h"], "encoded_height": padded(cfg["h"]), "frames": cfg["frames"],
           "content": cfg.get("content", "bench"), "vbs": bool(cfg.get("vbs")),
           "rate_control": ({"RCFlag": cfg["rc"], "target": cfg.get("target"), "roi": cfg.get("roi")}
                            if cfg.get("rc") else None)}
    if cfg.get("rc", 0) >= 3:   # configs[4]: the two-pass per-frame kernel sequence
        rec["roofline"] = rc_roofline(codec, frames, res["symbols"], args.kernel_reps, name)
    elif eng.pipelined_ok(1):   # right after timing, the GPU at its working clock
        rec["roofline"] = roofline_of(kernel_roofline(codec, frames, res["symbols"], args.kernel_reps,
                                                      components=False), name)
    if not cfg.get("rc"):
        rec["sea_dense_fallback"] = dense_fallback_of(eng, cfg, step)
    if not args.no_parity:
        def redo():
            poison(pre)
            r = step()
            eng.check_run()
            return r["symbols"]
        rec["parity"] = parity_of(res["symbols"], name, cfg, redo, sse=res["sse"])
    rec["roofline_gop"] = gop_roofline(cfg, elapsed / args.steps)
    rec["wait_health"] = eng.wait_health.as_dict()
    return rec


def record_gops_in_flight(name: str, ngops: int, args, dev) -> dict:
    """Throughput of a STREAM of GOPs: `ngops` independent GOPs of the workload per step
    (copies of its frames in separate buffers), their P-runs interleaved in one persistent
    launch (Y_Video_codec.encode_gops_device), so a frame of every GOP is in flight at once.
    One GOP's frame-to-frame dependency leaves CUs idle where a frame has fewer tiles than
    resident workgroups (1080p: 510 tiles, 768 slots); the other GOPs fill them.  Every GOP
    of the timed output is checked against the oracle fixture."""
    from streamoptima_amd.engine import alloc_planes
    from streamoptima_amd.workloads import WORKLOADS
    cfg = dict(WORKLOADS[name])
    codec = build_codec(cfg, args, dev)
    eng = codec.engine()
    src = make_frames(cfg, dev, cfg["seed"])
    gops = [src]
    for _ in range(ngops - 1):
        g = alloc_planes(*src.shape, dev)
        g.copy_(src)
        gops.append(g)
    f = cfg["frames"]
    pre = [[eng.new_symbols(0 if i % cfg["intra_dur"] == 0 else 1) for i in range(f)] for _ in gops]

    def step():
        return codec.encode_gops_device(gops, cfg["intra_dur"], symbols=pre, check=False)
    elapsed, res, runs = time_steps_median(step, args, dev)
    eng.check_run()
    mpx = args.steps * ngops * f * cfg["h"] * cfg["w"] / elapsed / 1e6
    rec = {"workload": f"{ngops} independent copies of {cfg['workload']} per step, P-runs interleaved in one "
                       "persistent launch (GOP-parallel stream encode)",
           "value": round(mpx, 2), "unit": "Mpx/s", "gops_per_step": ngops,
           "ms_per_step": round(elapsed / args.steps * 1e3, 3),
           "ms_per_gop": round(elapsed / args.steps / ngops * 1e3, 3), "ms_per_step_runs": runs}
    if not args.no_parity:
        per = [parity_of(r["symbols"], name, cfg, sse=r["sse"]) for r in res]
        rec["parity"] = {"bit_exact": all(p and p.get("bit_exact") for p in per),
                         "gops_checked": len(per), "fixture": per[0].get("fixture") if per[0] else None}
    rec["roofline_gop"] = gop_roofline(cfg, elapsed / args.steps, ngops)
    rec["wait_health"] = eng.wait_health.as_dict()
    return rec


# ---- multi-GPU hand-off -------------------------------------------------------------------------
def p2p_encoder(eng, frames, cfg, senc, world, max_wg=0, inject=False):
    """The in-launch stripe hand-off (streamoptima_amd/pipeline.py), self-checked before
    timing: the first 4 frames of the workload through it and through the RCCL all_gather
    path must give identical symbols on every rank, with no dependency wait timed out.
    Anything else (IPC unavailable, a lost flag, a mismatch) falls back to all_gather."""
    import torch.distributed as dist
    from streamoptima_amd.digest import frame_digest
    from streamoptima_amd.pipeline import PipelinedStripeGOPEncoder
    ok, penc, why = 1, None, ""
    try:
        penc = PipelinedStripeGOPEncoder(eng, cfg["frames"], max_wg=max_wg)
    except Exception as e:   # noqa: BLE001 -- any failure to set up the peer mapping
        ok, why = 0, f"setup: {e}"
    flag = torch.tensor([ok], dtype=torch.int32, device=eng.device)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if int(flag.item()) == 0:
        return None, "all_gather (RCCL) per frame; p2p hand-off unavailable" + (f" ({why})" if why else "")
    k = min(4, cfg["frames"])
    ok, why = 1, ""
    try:                      # this rank's launches only (see fpipe_encoder)
        a_syms = penc.r.encode(frames[:k], cfg["intra_dur"], cfg["qp"])
        torch.cuda.synchronize()
    except Exception as e:   # noqa: BLE001
        ok, why = 0, f"self-check run: {e}"
    flag = torch.tensor([ok], dtype=torch.int32, device=eng.device)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if int(flag.item()) == 0:
        return None, "all_gather (RCCL) per frame; p2p self-check run failed" + (f" ({why})" if why else "")
    b = senc.encode(frames[:k], cfg["intra_dur"], cfg["qp"])
    torch.cuda.synchronize()
    good = not penc.r.timed_out() and not inject    # inject: --inject-failure p2p_selfcheck
    for i in range(k):
        ga, gb = penc.gather_symbols(a_syms[i], i), senc.gather_symbols(b["symbols"][i])
        da = frame_digest(ga["frame_type"], {n: (v.cpu().numpy() if torch.is_tensor(v) else v) for n, v in ga.items()})
        db = frame_digest(gb["frame_type"], {n: (v.cpu().numpy() if torch.is_tensor(v) else v) for n, v in gb.items()})
        good = good and da == db
    flag = torch.tensor([1 if good else 0], dtype=torch.int32, device=eng.device)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if int(flag.item()) == 0:
        return None, "all_gather (RCCL) per frame; p2p self-check failed"
    return penc, "in-launch p2p over xGMI (uncached landing planes, IPC), self-checked"


def fpipe_rc_kw(codec) -> dict:
    """FramePipeRank.encode's rate-control keywords for the codec's RC / ROI settings (the
    row-QP schedule; RCFlag 3: two-pass with the ROI offsets and the QP clamp)."""
    eng = codec.engine()
    if not codec._rc_on():
        return {}
    kw = {"qp_row": codec.row_qp_schedule(eng.nby)}
    if codec.RCFlag >= 3:
        roi = codec.roi_block_offsets()
        kw.update(two_pass=True, roi_dev=eng.device_const_i32(roi) if roi is not None else None,
                  qp_clamp=tuple(codec.qp_clamp))
    return kw


def fpipe_encoder(codec, frames, cfg, world, max_wg=0, inject=False):
    """The frame pipeline (streamoptima_amd/pipeline.py FramePipelineGOPEncoder), self-checked
    before timing: the first 2N+1 frames through it must give, on every rank, the digests of
    a one-GPU encode of the same frames, with no hand-off wait timed out.  (None, why) else."""
    import torch.distributed as dist
    from streamoptima_amd.digest import symbols_digest
    from streamoptima_amd.pipeline import FramePipelineGOPEncoder
    eng = codec.engine()
    ok, penc, why = 1, None, ""
    if cfg["intra_dur"] < cfg["frames"] or not eng.pipelined_ok(1):
        ok, why = 0, "needs one I-frame per GOP and the persistent-run configuration"
    else:
        try:
            penc = FramePipelineGOPEncoder(eng, cfg["frames"], max_wg=max_wg)
        except Exception as e:   # noqa: BLE001 -- any failure to set up the peer mapping
            ok, why = 0, f"setup: {e}"
    flag = torch.tensor([ok], dtype=torch.int32, device=eng.device)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if int(flag.item()) == 0:
        return None, why or "unavailable on another rank"
    k = min(2 * world + 1, cfg["frames"])
    ok, why = 1, ""
    try:                      # this rank's launches only: a failure here must not strand the
        a = penc.encode_local(frames[:k], k, cfg["qp"], **fpipe_rc_kw(codec))   # other ranks in a collective
        torch.cuda.synchronize()
        ref = [symbols_digest(s) for s in codec.encode_device(frames[:k], k)["symbols"]]
    except Exception as e:   # noqa: BLE001
        ok, why = 0, f"self-check run: {e}"
    flag = torch.tensor([ok], dtype=torch.int32, device=eng.device)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if int(flag.item()) == 0:
        return None, why or "self-check run failed on another rank"
    got = penc.digests(a, k)
    good = not penc.r.timed_out() and got == ref and not inject   # inject: --inject-failure fpipe_selfcheck
    flag = torch.tensor([1 if good else 0], dtype=torch.int32, device=eng.device)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if int(flag.item()) == 0:
        from streamoptima_amd import runhealth
        runhealth.clear(penc.r._ws)
        return None, "self-check failed"
    return penc, "frame pipeline over xGMI (IPC-mapped uncached landing planes), self-checked"


# ---- CPU plumbing stand-in (--cpu-plumbing) ---------------------------------------------------------
class _PlumbingEngine:
    """A trivial CPU stand-in with the Engine stripe methods StripeGOPEncoder calls: symbols
    are zeros and the reconstruction is the source rows.  It encodes nothing; it only lets
    the rank launch, sharding, exchange, timing and JSON line run on a CPU-only host
    (tests/test_bench_dist.py)."""

    def __init__(self, h, w, bs=16):
        from streamoptima_amd.engine import Engine
        self.h, self.w, self.bs, self.sr = h, w, bs, 16
        self.nbx, self.nby = w // bs, h // bs
        self.nb = self.nbx * self.nby
        self.device = torch.device("cpu")
        self.new_stripe_symbols = Engine.new_stripe_symbols.__get__(self)

    def qp_row_tensor(self, q):
        return None if q is None else torch.tensor(list(q), dtype=torch.int32)

    def _rows(self, cur, by0, by1, out):
        for t in (out.split, out.mv, out.qtc, out.tokens, out.mae_num, out.sse):
            t.zero_()
        out.recon[by0 * self.bs:by1 * self.bs].copy_(cur[by0 * self.bs:by1 * self.bs])
        return out

    def encode_p_rows(self, cur, refs, by0, by1, qp, out, **kw):
        out.frame_type = 1
        return self._rows(cur, by0, by1, out)

    def encode_i_rows(self, cur, by0, by1, qp, out, **kw):
        out.frame_type = 0
        return self._rows(cur, by0, by1, out)


# ---- the printed line: compact, definitions stated once ------------------------------------------------
# the driver's parse failed on a 22.9 KB line (round 5; a 15.9 KB one parsed); its stdout tail keeps
# ~8 KB, so a line below that is whole even in the tail
LINE_MAX_BYTES = 7800
DEFS = {
    "algorithmic_bytes": ALG_BYTES_DEF,
    "frac": "required HBM fraction: algorithmic bytes per launch / average launch time (HIP events on the launch "
            "stream, this run) / 8 TB/s",
    "traffic": "HBM bytes per launch from separate rocprofv3 --pmc FETCH_SIZE (x2, tools/ubench_fetch.cpp) and "
               "WRITE_SIZE passes on the same workload: profiles/pmc_me_traffic.json, not this run",
    "valu_profile": "VALU busy fraction and waves/SIMD of the same kernel from the committed rocprofv3 --pmc "
                    "counters (profiles/pmc_me_traffic.json), not this run",
    "binding_limit": "the run kernel is bound by VALU issue (exact SEA search + FP64 pocketfft-exact DCT), not HBM",
    "sad_exec_frac": "executed v_sad_u8/v_sad_hi_u8 byte ops (counted in-kernel, one untimed replay) / run time / "
                     "measured v_sad peak 1.434e14 per s (tools/ubench_sad.cpp)",
    "parity": "per-frame sha256 of every symbol array + recon vs the C oracle's digests (tests/golden/large_gops.json); "
              "poisoned = one more step into 0xA5-filled outputs, compared again",
    "records": "other benchmarked configs at 1 GPU, each timed like the headline (median of --record-repeats runs)",
    "detail": "the uncompacted line (notes, per-field sources) is written to --detail-out",
}


def _pick(d, keys):
    return {k: d[k] for k in keys if isinstance(d, dict) and k in d}


def _compact_valu(v):
    if not v:
        return None
    return _pick(v, ("kernel", "valu_busy_frac", "waves_per_simd"))


def _compact_roofline(r, record=False):
    if not r or "error" in r:
        return r
    keys = (("kernel", "achieved", "frac", "traffic", "algorithmic_bytes", "per_frame_us") if record else
            ("bound", "kernel", "achieved", "peak", "unit", "frac", "traffic", "algorithmic_bytes", "launch_us",
             "frames_per_launch", "per_frame_us", "binding_limit"))
    out = _pick(r, keys)
    if "kernel" in out and out["kernel"].startswith("two-pass"):
        out["kernel"] = out["kernel"].split(": ", 1)[-1]
    vp = r.get("valu_profile") or r.get("valu")
    if vp:
        out["valu_profile"] = _compact_valu(vp)
    sad = r.get("sad") or {}
    if sad.get("executed_frac_of_measured_peak") is not None:
        out["sad_exec_frac"] = sad["executed_frac_of_measured_peak"]
    if not record and r.get("components"):
        out["components_us"] = {k: c.get("launch_us") for k, c in r["components"].items()}
    return out


def _compact_parity(p):
    if not p or "error" in p:
        return p
    out = _pick(p, ("bit_exact", "frames", "gops_checked", "psnr_delta_db", "poisoned_rerun_bit_exact"))
    if p.get("mismatched_frames"):
        out["mismatched_frames"] = p["mismatched_frames"]
    if p.get("note"):
        out["note"] = p["note"]
    return out


def _compact_health(h):
    if not h:
        return h
    out = _pick(h, ("timeouts", "stale_reads_repaired", "descheduled_polls"))
    if h.get("records"):
        out["first_record"] = h["records"][0]
    return out


def _compact_record(r):
    if not r or "error" in r:
        return r
    out = _pick(r, ("value", "ms_per_step", "ms_per_gop", "gops_per_step"))
    out["workload"] = r.get("workload", "")[:90]
    if r.get("roofline"):
        out["roofline"] = _compact_roofline(r["roofline"], record=True)
    if r.get("roofline_gop"):
        out["gop_frac"] = r["roofline_gop"].get("frac")
    if r.get("sea_dense_fallback"):
        out["dense_frac"] = r["sea_dense_fallback"].get("frac")
    if r.get("parity"):
        out["parity"] = _compact_parity(r["parity"])
    if r.get("wait_health"):
        out["wait_health"] = _compact_health(r["wait_health"])
    for k in r:
        if k not in out and k not in ("workload", "roofline", "roofline_gop", "sea_dense_fallback", "parity",
                                      "wait_health", "unit", "ms_per_step_runs", "width", "height", "encoded_height",
                                      "frames", "content", "vbs", "rate_control"):
            out[k] = r[k]
    return out


def compact_line(full: dict) -> dict:
    """The printed line: the full line with each shared definition stated once (`defs`) and
    every secondary entry cut to its numbers (the driver parses one line of bounded size;
    LINE_MAX_BYTES, tests/test_bench_line.py).  The full line goes to --detail-out."""
    line = {k: full[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                 "higher_is_better", "scaling", "vs_baseline", "dtype", "data") if k in full}
    cfg = dict(full.get("config") or {})
    line["config"] = _pick(cfg, ("workload", "name", "width", "height", "frames", "intra_dur", "block_size",
                                 "search_range", "qp", "seed", "vbs", "me", "content", "parallelism", "launch"))
    line["value_region"] = full.get("value_region")
    line["roofline"] = _compact_roofline(full.get("roofline"))
    cpu = full.get("cpu_baseline")
    if cpu:
        c = _pick(cpu, ("value", "unit", "cores", "kind", "sample", "host"))
        if "sample" in c:
            c["sample"] = c["sample"].split(", numpy port")[0] + ", numpy port of the reference loops (oracle/ref_numpy.py)"
        if cpu.get("pool"):
            c["pool"] = _pick(cpu["pool"], ("value", "cores"))
        if cpu.get("calibration"):
            c["port_over_reference_time"] = cpu["calibration"].get("port_over_reference_time")
        line["cpu_baseline"] = c
    else:
        line["cpu_baseline"] = cpu
    line["parity"] = _compact_parity(full.get("parity"))
    for k in ("psnr_mean_db", "psnr_delta_db", "gpu_over_cpu", "timeouts", "cpu_baseline_error", "degraded", "failed"):
        if k in full:
            line[k] = full[k]
    if full.get("roofline_gop"):
        line["gop_frac"] = full["roofline_gop"].get("frac")
    if full.get("sea_dense_fallback"):
        line["dense_frac"] = full["sea_dense_fallback"].get("frac")
    if "wait_health" in full:
        line["wait_health"] = _compact_health(full["wait_health"])
    s4 = full.get("section4_region")
    if s4:
        pc = full.get("pcie_inclusive") or {}
        rl = s4.get("roofline") or {}
        line["section4_region"] = {
            "value": s4.get("value"), "unit": s4.get("unit"), "ms_per_gop": s4.get("ms_per_gop"),
            "ms_per_gop_median": s4.get("ms_per_gop_median"),
            "roofline": {"bound": "pcie", "h2d_frac": rl.get("frac"), "achieved": rl.get("achieved"),
                         "peak": rl.get("peak"), "unit": "GB/s"},
            "packed_equals_resident_symbols": pc.get("packed_equals_resident_symbols"),
            "dense_ms_per_gop": (pc.get("dense") or {}).get("ms_per_gop")}
        for k in ("order_check",):
            if k in s4:
                line["section4_region"][k] = s4[k]
    elif full.get("pcie_inclusive") and "error" in full["pcie_inclusive"]:
        line["section4_region"] = full["pcie_inclusive"]
    if full.get("records"):
        line["records"] = {k: _compact_record(v) for k, v in full["records"].items()}
    line["defs"] = DEFS
    # never above the bound: shed the prose first, then the records' workload names
    if len(json.dumps(line)) > LINE_MAX_BYTES:
        line["defs"] = {"see": "bench.py DEFS"}
    if len(json.dumps(line)) > LINE_MAX_BYTES:
        for r in (line.get("records") or {}).values():
            if isinstance(r, dict):
                r.pop("workload", None)
    return line


# ---- main ----------------------------------------------------------------------------------------------
def main(argv=None):
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    world, rank, local = dist_setup("gloo" if (args.cpu_plumbing or args.share_gpu) else "nccl")
    if args.share_gpu:
        local = 0
        torch.cuda.set_device(0)
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}")
    from streamoptima_amd.workloads import WORKLOADS, variant_name
    name = variant_name(args.config or ("4k" if world == 1 else "4k120"), args.vbs, args.me)
    cfg = dict(WORKLOADS[name])
    if args.vbs:
        cfg["vbs"] = True
    if args.me != "full":
        cfg["me"] = args.me          # a mode without a fixture variant runs unchecked (parity None)
    if args.frames:
        cfg["frames"] = args.frames
        cfg["intra_dur"] = min(cfg["intra_dur"], args.frames)
    plain_cfg = cfg.get("me", "full") == "full" and not cfg.get("vbs")
    parity_ok = not (args.no_parity or args.frames)
    if args.shard is None:
        # two GPUs share ONE xGMI link: the frame pipeline would push every reconstruction
        # (8.3 MB per ~71 us frame, ~117 GB/s) over it one way, more than a link direction
        # carries, while two block-row stripes exchange 16-row halos and run 1,020 tiles each
        # at full throughput; from three ranks on the pipeline spreads over two links per
        # rank (alternating ring) and the stripes turn latency-bound
        args.shard = "stripe" if world == 2 else "fpipe"
    stripe = world > 1 and args.shard in ("stripe", "fpipe")    # one GOP over the ranks
    dev = torch.device("cpu") if args.cpu_plumbing else torch.device("cuda", local)
    h, w, f = cfg["h"], cfg["w"], cfg["frames"]

    exchange_note = "all_gather per frame"
    penc = fenc = None
    # a multi-GPU path that failed its self-check (or lost a hand-off in the timed run) and was
    # replaced by a fallback: the line still prints, names it under `degraded` and `failed`, and
    # the exit status is nonzero -- a fallback's time must never pass for the default path's
    degraded = []
    if args.cpu_plumbing and args.inject_failure in ("fpipe_selfcheck", "p2p_selfcheck"):
        degraded.append({"what": args.inject_failure, "why": f"--inject-failure {args.inject_failure}",
                         "timed_instead": "stripes, all_gather (RCCL) per frame"})
    mode_note = f"stripe x{world} (block rows of one GOP; hand-off: {{}})"
    if args.cpu_plumbing:
        from streamoptima_amd.dist import StripeGOPEncoder
        from streamoptima_amd.synth import synth_sequence
        from streamoptima_amd.workloads import padded
        eng = _PlumbingEngine(padded(h), padded(w))
        frames = torch.full((f, padded(h), padded(w)), 128, dtype=torch.uint8)
        frames[:, :h, :w] = torch.from_numpy(synth_sequence(f, h, w, seed=cfg["seed"]))
        senc = StripeGOPEncoder(eng)

        def step():
            return senc.encode(frames, cfg["intra_dur"], cfg["qp"])
        codec = None
    elif stripe:
        from streamoptima_amd.dist import StripeGOPEncoder
        codec = build_codec(cfg, args, dev)
        eng = codec.engine()
        frames = make_frames(cfg, dev, cfg["seed"])
        senc = StripeGOPEncoder(eng)
        rc = cfg.get("rc")
        cap = 768 // (2 * world) if args.share_gpu else 0
        plain = not rc and plain_cfg and eng.pipelined_ok(1, vbs_ok=False)
        # the frame pipeline covers the plain GOP, VBSEnable and two-pass RC / ROI (configs[4]):
        # a rank owns whole frames, so the row-local QP statistics never cross ranks
        fp_ok = cfg.get("me", "full") == "full" and eng.pipelined_ok(1) and (
            not rc or (rc >= 3 and codec.intra_thresh is None and not cfg.get("vbs")))
        fpipe_note = ""
        if args.shard == "fpipe" and fp_ok:
            fenc, fpipe_note = fpipe_encoder(codec, frames, cfg, world, max_wg=cap,
                                             inject=args.inject_failure == "fpipe_selfcheck")
            if fenc is None:
                degraded.append({"what": "fpipe_selfcheck", "why": fpipe_note,
                                 "timed_instead": "block-row stripes" + (" (p2p hand-off)" if plain and
                                                                          args.exchange == "p2p" else "")})
        if fenc is not None:
            mode_note = (f"frame pipeline x{world} (one frame per rank per block of N frames, ring direction "
                         f"alternating per block; {{}})")
            exchange_note = fpipe_note

            # the SSE all_reduce runs once, after timing (pipeline.py encode), unless every rank
            # does not hold a P-frame (frames <= ranks): then it orders back-to-back GOPs
            b2b = f > world
            rc_kw = fpipe_rc_kw(codec)

            def step():
                return fenc.encode(frames, cfg["intra_dur"], cfg["qp"], reduce=not b2b, **rc_kw)
        else:
            if args.exchange == "p2p" and plain:
                penc, exchange_note = p2p_encoder(eng, frames, cfg, senc, world, max_wg=cap,
                                                  inject=args.inject_failure == "p2p_selfcheck")
                if penc is None:
                    degraded.append({"what": "p2p_selfcheck", "why": exchange_note,
                                     "timed_instead": "stripes, all_gather (RCCL) per frame"})
            else:
                exchange_note = "all_gather (RCCL) per frame" + (": RC/ROI GOP" if rc else "")
            if fpipe_note:
                exchange_note += f"; frame pipeline not used: {fpipe_note}"
            if penc is not None:
                pre_s = [penc.r.new_symbols(0 if i % cfg["intra_dur"] == 0 else 1) for i in range(f)]

                def step():
                    return penc.encode(frames, cfg["intra_dur"], cfg["qp"], symbols=pre_s)
            else:
                def step():
                    return senc.encode(frames, cfg["intra_dur"], cfg["qp"],
                                       qp_sched=codec.row_qp_schedule(eng.nby) if rc else None, rc_flag=rc,
                                       intra_thresh=None, roi=codec.roi_block_offsets())
    else:
        codec, frames, pre, step = run_single(cfg, args, dev, parity_ok)
        if world > 1 and rank > 0:   # --shard gop: an independent GOP per rank (seed + rank)
            frames.copy_(make_frames(cfg, dev, cfg["seed"] + rank))

    elapsed, res = time_steps(step, world, args.steps, args.warmup, dev)
    if codec is not None and not stripe:
        codec.engine().check_run()
    timeouts = None
    if penc is not None or fenc is not None:
        # a lost hand-off anywhere voids the timed run: time the all_gather path instead
        import torch.distributed as dist
        from streamoptima_amd import runhealth
        r_ = (penc or fenc).r
        h_ = runhealth.read(r_._ws)
        if h_["record"]:
            print(f"bench.py rank {rank}: hand-off wait timed out: {runhealth.describe(h_['record'])}",
                  file=sys.stderr, flush=True)
        lost = torch.tensor([h_["timeouts"]], dtype=torch.int32, device=dev)
        dist.all_reduce(lost, op=dist.ReduceOp.SUM)
        timeouts = int(lost.item())
        if timeouts:
            degraded.append({"what": "handoff_timeout", "why": f"{timeouts} in-launch hand-off wait(s) timed out in "
                             "the timed run, which was discarded", "timed_instead": "stripes, all_gather (RCCL) per frame"})
            runhealth.clear(r_._ws)
            penc = fenc = None
            mode_note = f"stripe x{world} (block rows of one GOP; hand-off: {{}})"
            exchange_note = "all_gather (RCCL) per frame; the p2p run timed out a hand-off and was discarded"

            def step():  # noqa: F811
                return senc.encode(frames, cfg["intra_dur"], cfg["qp"])
            elapsed, res = time_steps(step, world, args.steps, args.warmup, dev)

    # ---- right after timing (GPU still at its working clock): the dominant kernel's roofline ----
    rl = None
    if (rank == 0 and not args.cpu_plumbing and cfg.get("me", "full") == "full" and codec.engine().pipelined_ok(1)
            and not cfg.get("rc")):
        # stripe mode: the kernel is timed on rank 0's GPU alone over the full frame (a
        # one-GPU GOP supplies the reference reconstructions it replays)
        syms = res["symbols"] if not stripe else codec.encode_device(frames, cfg["intra_dur"])["symbols"]
        rl = kernel_roofline(codec, frames, syms, args.kernel_reps, components=not cfg.get("vbs"))
    rl_rc = None
    if rank == 0 and not args.cpu_plumbing and cfg.get("rc", 0) >= 3 and not stripe and codec.engine().pipelined_ok(1):
        rl_rc = rc_roofline(codec, frames, res["symbols"], args.kernel_reps, name)

    # ---- after timing: parity of the timed output ----
    parity = None
    if parity_ok and not args.cpu_plumbing:
        if fenc is not None:
            fenc.check()
            res["sse"] = fenc.sse(res["symbols"], f)
            got = fenc.digests(res["symbols"], f)
            if rank == 0:
                fx = load_fixture(name)
                parity = compare_digests(got, fx) if fx else {"bit_exact": None, "note": "no fixture"}
                if fx:
                    parity["fixture"] = "tests/golden/large_gops.json (C oracle, tests/golden/make_large_fixtures.py)"
                    parity["psnr_delta_db"] = psnr_delta(res["sse"], fx, -(-h // 16) * 16, w)["psnr_delta_db_max"]
        elif stripe:
            if penc is not None:
                penc.check()
                full = [penc.gather_symbols(s, i) for i, s in enumerate(res["symbols"])]
            else:
                full = [senc.gather_symbols(s) for s in res["symbols"]]
            if rank == 0:
                hosts = [{k: (v.cpu().numpy() if torch.is_tensor(v) else v) for k, v in g.items()} for g in full]
                parity = parity_of(hosts, name, cfg, sse=res["sse"])
        elif rank == 0 or world == 1:
            def redo():
                poison(pre)
                r = step()
                codec.engine().check_run()
                return r["symbols"]
            parity = parity_of(res["symbols"], name, cfg, redo, sse=res["sse"])
    barrier(world)

    fallback = None
    if (world == 1 and not args.cpu_plumbing and codec is not None and cfg.get("me", "full") == "full"
            and not cfg.get("rc") and codec.engine().pipelined_ok(1)):
        fallback = dense_fallback_of(codec.engine(), cfg, step)

    psnr_mean = None
    if "sse" in res:
        hp = -(-h // 16) * 16
        sse = res["sse"].cpu().numpy()
        vals = [10 * np.log10(255 ** 2 / (s / (hp * w))) for s in sse if s > 0]
        psnr_mean = float(np.mean(vals)) if vals else None

    # ---- secondary measurements: each one's failure is recorded in the line (and makes the exit
    # status nonzero) instead of voiding the headline measured above ----
    failures = []

    def guarded(what, fn):
        try:
            if args.inject_failure == what:
                raise RuntimeError(f"--inject-failure {what}")
            return fn()
        except Exception as e:   # noqa: BLE001 -- reported, never swallowed: rc != 0 below
            import traceback
            failures.append(what)
            print(f"bench.py: {what} failed:\n{traceback.format_exc()}", file=sys.stderr, flush=True)
            return {"error": f"{type(e).__name__}: {e}"}

    headline_health = None
    if codec is not None and not stripe:
        headline_health = codec.engine().wait_health.as_dict()
    # BASELINE.md section 4's region first, right after the headline (a run of records ahead of it
    # left the region 1.6x slower on one box: profiles/r05/pcie_order.log)
    pcie = None
    if rank == 0 and world == 1 and not args.cpu_plumbing and not args.no_pcie and plain_cfg and not args.pcie_last:
        pcie = guarded("pcie_inclusive", lambda: pcie_inclusive(codec, cfg, frames))
    records = None
    if rank == 0 and world == 1 and not args.cpu_plumbing and not args.no_records and name == "4k":
        records = {"1080p": guarded("records.1080p", lambda: record_single("1080p", args, dev))}
        for k in args.gops_in_flight:
            for nm in ("1080p", "4k"):
                records[f"{nm}_x{k}gop"] = guarded(f"records.{nm}_x{k}gop",
                                                   lambda nm=nm, k=k: record_gops_in_flight(nm, k, args, dev))
        if not args.no_content_records:
            for nm in ("4k_lowtex", "4k_noise"):
                records[nm] = guarded(f"records.{nm}", lambda nm=nm: record_single(nm, args, dev))
        # the other benchmarked settings of configs[2] / configs[4] at one GPU: VBSEnable and the
        # ROI + two-pass rate-control GOP, each measured and parity-checked like the headline
        for nm in ("4k_vbs", "4k_rc2pass"):
            records[nm] = guarded(f"records.{nm}", lambda nm=nm: record_single(nm, args, dev))
    if rank == 0 and world == 1 and not args.cpu_plumbing and not args.no_pcie and plain_cfg and args.pcie_last:
        pcie = guarded("pcie_inclusive", lambda: pcie_inclusive(codec, cfg, frames))
    if rank == 0 and args.cpu_plumbing and args.inject_failure and not any(
            d["what"] == args.inject_failure for d in degraded):   # the mechanism, on a CPU-only host
        records = {args.inject_failure: guarded(args.inject_failure, lambda: {"plumbing": True})}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.cpu_plumbing:
        cpu = guarded("cpu_baseline", lambda: cpu_baseline(cfg, args.cpu_rows, args.cpu_pool_rows))
    if rank != 0:
        barrier(world)
        return
    ms_per_step = elapsed / args.steps * 1e3
    units = 1 if (stripe or args.cpu_plumbing) else world   # GOPs encoded per step across the job
    mpx = units * args.steps * f * h * w / elapsed / 1e6
    line = {
        "metric": METRIC,
        "value": round(mpx, 2), "unit": "Mpx/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
        "scaling": "strong" if (stripe or args.cpu_plumbing) else "weak",
        "vs_baseline": None, "dtype": "u8",
        "value_region": "hbm_resident",
        "value_region_note": ("value: frames already resident in HBM when the timed region starts (the task's "
                              "measurement contract); BASELINE.md section 4's region (pinned host Y planes in, "
                              "symbols out over PCIe) is section4_region, measured in the same run"),
        "data": ("plumbing self-test: trivial CPU stand-in engine, nothing encoded" if args.cpu_plumbing else
                 "synthetic (splitmix64 texture, +2/+1 px/frame motion, streamoptima_amd/synth.py)"),
        "config": {"workload": cfg["workload"], "name": name, "width": w, "height": h, "frames": f,
                   "intra_dur": cfg["intra_dur"], "block_size": 16, "search_range": 16, "qp": cfg["qp"],
                   "seed": cfg["seed"], "vbs": bool(cfg.get("vbs")), "nRefFrames": 1, "me": cfg.get("me", "full"),
                   "content": cfg.get("content", "bench"),
                   "transform": "fp64 pocketfft-exact DCT",
                   "parallelism": (mode_note.format(exchange_note) if stripe else f"gop-per-rank x{world}"),
                   "launch": ("hip-graph (one GOP per replay)" if (args.graph and not stripe and not args.cpu_plumbing)
                              else "host launches")},
        "parity": parity,
        "roofline": roofline_of(rl, name) if rl else rl_rc,
        "roofline_gop": gop_roofline(cfg, elapsed / args.steps) if (world == 1 and not args.cpu_plumbing) else None,
        "cpu_baseline": cpu if (cpu is None or "error" not in cpu) else None,
        "psnr_mean_db": round(psnr_mean, 4) if psnr_mean is not None else None,
        "psnr_delta_db": parity.get("psnr_delta_db") if parity else None,
    }
    if fallback:
        line["sea_dense_fallback"] = fallback
    if world > 1:
        # dependency waits of the in-launch hand-off that passed their bound during the timed
        # run, summed over ranks (nonzero: that run was discarded and the stripes timed instead)
        line["timeouts"] = timeouts
    if headline_health is not None:
        line["wait_health"] = headline_health
    if records:
        line["records"] = records
    if pcie:
        line["pcie_inclusive"] = pcie
        if "error" not in pcie:
            line["section4_region"] = {
                "region": "BASELINE.md section 4: host-pinned Y planes -> HBM, the GOP encode, the symbols back to "
                          "pinned host memory (packed stream + per-frame SSE)",
                "value": pcie["mpx_s"], "unit": "Mpx/s", "ms_per_gop": pcie["ms_per_gop"],
                "ms_per_gop_median": pcie["ms_per_gop_median"], "roofline": pcie["roofline"],
                "detail": "pcie_inclusive"}
    if cpu and cpu.get("value"):
        line["gpu_over_cpu"] = round(mpx / cpu["value"], 1)
    if cpu and "error" in cpu:
        line["cpu_baseline_error"] = cpu["error"]
    if degraded:
        line["degraded"] = degraded
        failures.extend(d["what"] for d in degraded)
    if failures:
        line["failed"] = failures
    if args.detail_out:   # '' = nowhere
        try:
            os.makedirs(os.path.dirname(os.path.abspath(args.detail_out)), exist_ok=True)
            with open(args.detail_out, "w") as fh:
                json.dump(line, fh, indent=1)
        except OSError as e:
            print(f"bench.py: --detail-out {args.detail_out}: {e}", file=sys.stderr, flush=True)
    print(json.dumps(compact_line(line)), flush=True)
    barrier(world)
    if failures:
        sys.exit(f"bench.py: {len(failures)} measurement(s) failed or degraded: {', '.join(failures)} "
                 "(the line above is complete; `degraded` names a multi-GPU fallback that was timed instead)")



if __name__ == "__main__":
    main()
