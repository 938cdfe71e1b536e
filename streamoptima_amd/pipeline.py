"""ONE GOP across the GPUs of a node with the hand-off inside the persistent launch
(BASELINE configs[3]).

Encoder.encode() (reference Encoder.py:1790-1898) is sequential over frames: P(i) searches
the reconstruction of frame i-1 (:1864-1867).  Its blocks are independent given that
reference, and a block's +-16 px search window reaches only the neighbouring block rows, so:

  * rank r of N owns the block rows [by0, by1) of every frame (dist.stripe_rows);
  * one persistent launch per <= 32 P-frames runs the rank's stripe of consecutive frames
    (so_encode_p_run_stripe): a tile of frame f starts once the tiles of frame f-1 its
    window reads are done -- its own rank's 3x3 neighbourhood, and for the stripe's first /
    last tile row also the neighbour rank's three tiles across the boundary;
  * those neighbour tiles store their 16 boundary rows straight into this rank's uncached
    landing plane of the frame (peer memory over xGMI, mapped by IPC) and raise a flag there,
    so frames pipeline across the ranks exactly as they do across the workgroups of one GPU:
    no host round trip and no collective per frame;
  * the I-frame's stripe (intra mode 0 needs no halo) is followed by one small push of its
    boundary rows (so_stripe_halo_push).

The symbols are the rank-order concatenation of the stripes, bit-identical to one GPU.  The
per-row RC schedule is content-independent (:1599-1609) but this path runs the plain GOP
(configs[3]); RC / ROI / two-pass GOPs use dist.StripeGOPEncoder.

`StripeRunRank` holds one rank's buffers and launches; `connect()` takes the neighbours'
buffers as mapped in this process (IPC handles across processes, plain pointers when several
ranks share one GPU in the tests).  `PipelinedStripeGOPEncoder` is the torch.distributed
front end (handles exchanged with all_gather_object; SSE summed with one all_reduce).
"""
from __future__ import annotations

import contextlib
import ctypes
import weakref

import torch

from . import _lib, runhealth
from .dist import stripe_rows
from .engine import FrameSymbols

HALO_TOP, HALO_BOT = 16, 32       # landing-plane rows above / below the stripe

# Resident-slot claims of the ranks living in THIS process, per device (DESIGN.md section 6,
# "Forward progress"): a rank's persistent launch may wait on another rank's tasks, which only
# a resident workgroup of that rank's launch can take.  One rank per GPU always fits (each
# launch's grid is at most its device's resident capacity).  Ranks sharing one device (the
# in-process tests, --share-gpu rehearsals) must cap their grids (max_wg) so that every
# launch can be resident at once -- in practice with a margin: three two-pass ranks whose grids
# summed to exactly the device's capacity stalled (profiles/r03/fpipe2p_fullcap_w3.log), while
# three quarters of it has always run -- so ranks sharing a device may together claim that.  A
# rank whose claim would overflow it is refused here instead of stalling its peers until the
# wait bound.
_CLAIMS: dict = {}
SHARED_LIMIT = 0.75


def _claim_slots(owner, engine, max_wg: int, vbs: bool):
    """Record this rank's resident-slot claim on its device (the fraction of the device's
    resident workgroups its launch grid takes); refuse it if the device would be overcommitted."""
    dev = engine.device.index if engine.device.index is not None else torch.cuda.current_device()
    with torch.cuda.device(dev):
        cap = _lib.load().so_p_run_resident_workgroups(int(vbs))
    if cap <= 0:
        _lib.check(cap, "so_p_run_resident_workgroups")
    want = max_wg if 0 < max_wg <= cap else cap
    frac = want / cap
    live = _CLAIMS.setdefault(dev, {})

    def limit():   # a lone rank: the whole device; ranks sharing it: SHARED_LIMIT of it together
        return 1.0 if not live else SHARED_LIMIT
    held = sum(live.values())
    if held + frac > limit() + 1e-9:
        import gc
        gc.collect()   # ranks already dropped but held by a reference cycle release their claims
        held = sum(live.values())
    if held + frac > limit() + 1e-9:
        raise ValueError(f"{type(owner).__name__}: {len(live)} rank(s) of this process already hold {held:.2f} of the "
                         f"resident workgroups of cuda:{dev}; this rank's run needs {want} of {cap} (max_wg "
                         f"{max_wg or 'uncapped'}). Ranks sharing one GPU must cap max_wg so that their launches "
                         f"together use at most {SHARED_LIMIT:.0%} of it (DESIGN.md section 6, forward progress)")
    key = id(owner)
    live[key] = frac
    owner._claim = (dev, key)
    weakref.finalize(owner, live.pop, key, None)
    return want


def _release_slots(owner) -> None:
    dev, key = getattr(owner, "_claim", (None, None))
    if dev is not None:
        _CLAIMS.get(dev, {}).pop(key, None)


class StripeRunRank:
    """Buffers and launches of one rank of a GOP split into block-row stripes."""

    def __init__(self, engine, world: int, rank: int, max_frames: int, stream=None, max_wg: int = 0):
        e = engine
        if not e.pipelined_ok(1, vbs_ok=False):
            raise ValueError("the stripe run covers bs 16 / sr 16 / full search / no VBS, FME / W % 128 == 0")
        self.eng, self.world, self.rank = e, world, rank
        self.by0, self.by1, self.rps = stripe_rows(e.nby, world, rank)
        if self.by1 <= self.by0:
            raise ValueError(f"rank {rank} of {world} has no block rows ({e.nby} rows)")
        self.max_frames = max_frames
        self.stream = stream
        self.max_wg = max_wg
        self.resident = _claim_slots(self, e, max_wg, False)
        self.tiles_x = e.w // 128
        lib = self.lib = _lib.load()
        w = e.w
        self.ext_rows = self.rps * 16 + HALO_TOP + HALO_BOT
        self.stride = -(-self.ext_rows * w // 256) * 256
        self._planes = ctypes.c_void_p()
        _lib.check(lib.so_alloc_uncached(max_frames * self.stride + 256, ctypes.byref(self._planes)), "so_alloc_uncached")
        self._flags = ctypes.c_void_p()
        self.flag_words = 2 * max_frames * self.tiles_x
        _lib.check(lib.so_alloc_uncached(self.flag_words * 4, ctypes.byref(self._flags)), "so_alloc_uncached")
        _lib.check(lib.so_memset_d8(self._flags, 0, self.flag_words * 4, self._st()), "so_memset_d8")
        _lib.check(lib.so_memset_d8(self._planes, 0, max_frames * self.stride + 256, self._st()), "so_memset_d8")
        self.epoch = 0
        self.peer_up = self.peer_dn = None      # (virtual base of frame 0, flags array to set)
        self._opened = []
        self._ws = torch.zeros(lib.so_p_run_workspace_elems(e.h, e.w), dtype=torch.int32, device=e.device)
        self.wait_health = runhealth.HealthLog()

    # ---- addressing -----------------------------------------------------------------------
    def _st(self):
        return self.stream.cuda_stream if self.stream is not None else _lib.stream_handle(self.eng.device)

    @property
    def planes(self) -> int:
        return self._planes.value

    @property
    def flags(self) -> int:
        return self._flags.value

    def up_flags(self) -> int:       # set by the up neighbour (its bottom rows arrived)
        return self.flags

    def dn_flags(self) -> int:       # set by the down neighbour
        return self.flags + self.max_frames * self.tiles_x * 4

    def virt(self, gf: int, planes: int | None = None, by0: int | None = None) -> int:
        """Virtual full-frame base of frame gf's landing plane (row y at base + y * W)."""
        planes = self.planes if planes is None else planes
        by0 = self.by0 if by0 is None else by0
        return planes + gf * self.stride - (by0 * 16 - HALO_TOP) * self.eng.w

    def info(self) -> dict:
        """What a neighbour needs to reach this rank (pointers valid in THIS process)."""
        return {"planes": self.planes, "flags": self.flags, "by0": self.by0, "rank": self.rank}

    def export(self) -> dict:
        """IPC handles of this rank's planes and flags (for another process)."""
        hp = (ctypes.c_uint8 * 64)()
        hf = (ctypes.c_uint8 * 64)()
        _lib.check(self.lib.so_ipc_export(self._planes, hp), "so_ipc_export")
        _lib.check(self.lib.so_ipc_export(self._flags, hf), "so_ipc_export")
        return {"planes_h": bytes(hp), "flags_h": bytes(hf), "by0": self.by0, "rank": self.rank}

    def open(self, exported: dict) -> dict:
        """Map a neighbour's exported buffers into this process."""
        out = {"by0": exported["by0"], "rank": exported["rank"]}
        for k in ("planes", "flags"):
            p = ctypes.c_void_p()
            h = (ctypes.c_uint8 * 64).from_buffer_copy(exported[k + "_h"])
            _lib.check(self.lib.so_ipc_open(h, ctypes.byref(p)), "so_ipc_open")
            self._opened.append(p)
            out[k] = p.value
        return out

    def connect(self, up: dict | None, dn: dict | None) -> None:
        """up / dn: the neighbours' info() as mapped in this process (None at the frame edge)."""
        mf, tx = self.max_frames, self.tiles_x
        if up is not None:
            # my top rows land in the up neighbour's plane below ITS stripe; its dn flags
            self.peer_up = (self.virt(0, up["planes"], up["by0"]), up["flags"] + mf * tx * 4)
        if dn is not None:
            self.peer_dn = (self.virt(0, dn["planes"], dn["by0"]), dn["flags"])

    def close(self) -> None:
        for p in self._opened:
            self.lib.so_ipc_close(p)
        self._opened = []
        for p in (self._planes, self._flags):
            if p.value:
                self.lib.so_free_device(p)
        self._planes = ctypes.c_void_p()
        self._flags = ctypes.c_void_p()
        _release_slots(self)

    # ---- one GOP ---------------------------------------------------------------------------
    def new_symbols(self, frame_type: int) -> FrameSymbols:
        e, bs = self.eng, self.eng.bs
        d = e.device
        nbs = e.nbx * (self.by1 - self.by0)
        mv_shape = (nbs, 4, 3) if frame_type == 1 else (nbs, 4)
        return FrameSymbols(frame_type=frame_type,
                            split=torch.empty(nbs, dtype=torch.uint8, device=d),
                            mv=torch.empty(mv_shape, dtype=torch.int16, device=d),
                            qtc=torch.empty((nbs, bs * bs), dtype=torch.int16, device=d),
                            tokens=torch.empty(nbs, dtype=torch.int32, device=d),
                            mae_num=torch.empty(nbs, dtype=torch.int32, device=d),
                            recon=None,
                            sse=torch.zeros(max(nbs, (self.by1 - self.by0) * bs), dtype=torch.int32, device=d),
                            extra={"by0": self.by0, "by1": self.by1})

    def encode(self, frames: torch.Tensor, intra_dur: int, qp: int, out=None) -> list:
        """The stripe's symbols of every frame (stripe-local; recon stays in the landing
        planes: stripe_recon(gf)).  Asynchronous on the rank's stream; no host sync."""
        e, lib = self.eng, self.lib
        nf = frames.shape[0]
        if nf > self.max_frames:
            raise ValueError(f"{nf} frames > max_frames {self.max_frames}")
        self.epoch += 1
        ep = self.epoch
        st = self._st()
        syms = out if out is not None else [self.new_symbols(0 if i % intra_dur == 0 else 1) for i in range(nf)]
        up_v, up_f = self.peer_up if self.peer_up else (None, None)
        dn_v, dn_f = self.peer_dn if self.peer_dn else (None, None)
        my_up = self.up_flags() if self.peer_up else None
        my_dn = self.dn_flags() if self.peer_dn else None
        i = 0
        while i < nf:
            if i % intra_dur == 0:
                s = syms[i]
                _lib.check(lib.so_encode_i_rows_ex(
                    frames[i].data_ptr(), e.h, e.w, e.bs, e.sr, self.by0, self.by1, int(qp), None, None, 0, 0.0,
                    s.split.data_ptr(), s.mv.data_ptr(), s.qtc.data_ptr(), s.tokens.data_ptr(), s.mae_num.data_ptr(),
                    self.virt(i), s.sse.data_ptr(), e.scratch.data_ptr(), st), "so_encode_i_rows_ex")
                s.frame_type, s.qp_rd = 0, int(qp)
                _lib.check(lib.so_stripe_halo_push(
                    self.virt(i), e.h, e.w, self.by0, self.by1, i,
                    None if up_v is None else up_v + i * self.stride, None if dn_v is None else dn_v + i * self.stride,
                    up_f, dn_f, ep, st), "so_stripe_halo_push")
                i += 1
                continue
            j = i
            while j < nf and j % intra_dur != 0:
                j += 1
            n = j - i
            arr = lambda xs: (ctypes.c_void_p * n)(*xs)  # noqa: E731
            ss = syms[i:j]
            _lib.check(lib.so_encode_p_run_stripe(
                arr([frames[k].data_ptr() for k in range(i, j)]), n, self.virt(i - 1), e.h, e.w, e.bs, e.sr,
                self.by0, self.by1, int(qp), None,
                arr([s.split.data_ptr() for s in ss]), arr([s.mv.data_ptr() for s in ss]),
                arr([s.qtc.data_ptr() for s in ss]), arr([s.tokens.data_ptr() for s in ss]),
                arr([s.mae_num.data_ptr() for s in ss]), arr([self.virt(k) for k in range(i, j)]),
                arr([s.sse.data_ptr() for s in ss]), self._ws.data_ptr(), i,
                up_v, dn_v, self.stride, my_up, my_dn, up_f, dn_f, ep, int(self.max_wg), st), "so_encode_p_run_stripe")
            for s in ss:
                s.frame_type, s.qp_rd = 1, int(qp)
            i = j
        return syms

    def stripe_recon(self, gf: int) -> torch.Tensor:
        """The stripe's rows of frame gf's reconstruction, copied into a tensor."""
        e = self.eng
        rows = (self.by1 - self.by0) * 16
        out = torch.empty((rows, e.w), dtype=torch.uint8, device=e.device)
        src = self.virt(gf) + self.by0 * 16 * e.w
        # on the caller's stream (which `out` belongs to), after everything on the rank's
        cur = torch.cuda.current_stream(e.device)
        if self.stream is not None:
            cur.wait_stream(self.stream)
        _lib.check(self.lib.so_copy_d2d(out.data_ptr(), src, rows * e.w, cur.cuda_stream), "so_copy_d2d")
        return out

    def timed_out(self) -> bool:
        return runhealth.timed_out(self._ws)

    def check(self) -> None:
        """Raise (naming the first timed-out wait: peer flags, slot, epoch) if a hand-off wait
        timed out since the last check; clear the counts."""
        runhealth.check(self._ws, self.wait_health, "p_run stripe (hand-off)")


class PipelinedStripeGOPEncoder:
    """torch.distributed front end of StripeRunRank: one rank per GPU, neighbours' buffers
    mapped by IPC (handles exchanged with all_gather_object over the process group)."""

    def __init__(self, engine, max_frames: int, group=None, max_wg: int = 0):
        import torch.distributed as dist
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.eng = engine
        self.r = StripeRunRank(engine, self.world, self.rank, max_frames, max_wg=max_wg)
        torch.cuda.synchronize(engine.device)
        if self.world > 1:
            mine = self.r.export()
            alls = [None] * self.world
            dist.all_gather_object(alls, mine, group=group)
            # ranks past the last block row own nothing (never happens for world <= nby)
            up = self.r.open(alls[self.rank - 1]) if self.rank > 0 else None
            dn = self.r.open(alls[self.rank + 1]) if self.rank < self.world - 1 else None
            self.r.connect(up, dn)
            dist.barrier(group=group)
        self.by0, self.by1, self.rps = self.r.by0, self.r.by1, self.r.rps

    def encode(self, frames, intra_dur: int, qp: int, symbols=None) -> dict:
        syms = self.r.encode(frames, intra_dur, qp, out=symbols)
        sse = torch.stack([s.sse for s in syms]).sum(dim=1, dtype=torch.int64)
        if self.world > 1:
            import torch.distributed as dist
            dist.all_reduce(sse, group=self.group)
        return {"symbols": syms, "frame_type": [s.frame_type for s in syms], "sse": sse}

    def check(self) -> None:
        self.r.check()

    def gather_symbols(self, sym, gf: int) -> dict:
        """Whole-frame symbols of frame gf (rank-order concatenation) on every rank."""
        import torch.distributed as dist
        e = self.eng
        nbx, rows = e.nbx, self.rps * 16
        out = {}
        for name in ("split", "mv", "qtc", "tokens", "mae_num"):
            t = getattr(sym, name)
            rec = tuple(t.shape[1:])
            pad = torch.zeros((self.rps * nbx,) + rec, dtype=t.dtype, device=t.device)
            pad[: t.shape[0]].copy_(t)
            full = torch.empty((self.world * self.rps * nbx,) + rec, dtype=t.dtype, device=t.device)
            if self.world > 1:
                dist.all_gather_into_tensor(full.view(-1).view(torch.uint8), pad.view(-1).view(torch.uint8),
                                            group=self.group)
            else:
                full.copy_(pad)
            out[name] = full[: e.nby * nbx]
        rec = torch.zeros((rows, e.w), dtype=torch.uint8, device=e.device)
        mine = self.r.stripe_recon(gf)
        rec[: mine.shape[0]].copy_(mine)
        full = torch.empty((self.world * rows, e.w), dtype=torch.uint8, device=e.device)
        if self.world > 1:
            dist.all_gather_into_tensor(full.view(-1), rec.view(-1), group=self.group)
        else:
            full.copy_(rec)
        out["recon"] = full[: e.h]
        out["frame_type"] = sym.frame_type
        return out

    def close(self) -> None:
        self.r.close()


# ---- frame pipeline: consecutive frames on consecutive ranks -----------------------------------
def fpipe_rank_of(world: int, f: int) -> int:
    """The rank encoding frame f: blocks of `world` consecutive frames are dealt to the ranks in
    alternating ring directions -- block k even: position i -> rank i; odd: rank (-i) mod N --
    so frame f + 1 is on rank(f) + 1 in even blocks and rank(f) - 1 in odd ones (across a
    block boundary too): every rank hands its reconstructions alternately to its two ring
    neighbours, and both directions of every xGMI link carry half the frames."""
    k, i = divmod(f, world)
    return i if k % 2 == 0 else (world - i) % world


def fpipe_plan(world: int, rank: int, nframes: int) -> dict:
    """Which frames rank `rank` of `world` encodes and where its references land.
    frames: its global frame indices, one per block of `world` frames (slot j <-> block j);
    run: the P-frames of its persistent launch (rank 0's frame 0 is the I-frame); slot0: the
    slot of run[0] (its reference, frame run[0] - 1, arrives in that landing slot); push: per
    run frame f, where frame f's reconstruction goes -- slot (f + 1) // world of rank
    fpipe_rank_of(f + 1), coded slot * 2 + (0: the next rank, 1: the previous rank), or -1 for
    the GOP's last frame (nothing reads it: no push over the link)."""
    nblocks = -(-nframes // world)
    frames = []
    for k in range(nblocks):
        f = k * world + (rank if k % 2 == 0 else (world - rank) % world)
        if f < nframes:
            frames.append(f)
    run = [k for k in frames if k > 0]
    push = []
    for f in run:
        if f + 1 >= nframes:      # the GOP's last frame: no rank reads its reconstruction
            push.append(-1)
            continue
        r = fpipe_rank_of(world, f + 1)
        if r not in ((rank + 1) % world, (rank - 1) % world):
            raise AssertionError("fpipe_plan: frame f + 1 is not on a ring neighbour")
        push.append(((f + 1) // world) * 2 + (0 if r == (rank + 1) % world else 1))
    return {"frames": frames, "run": run, "slot0": run[0] // world if run else 0, "push": push,
            "nslots": nblocks + 1}


def fpipe_p2lag(world: int, ntr: int) -> int:
    """Cap on the pass-2 lag (tile rows) of the two-pass frame pipeline, 0 = no cap.  The
    library queues a tile row's pass-2 tasks about one grid's worth of rows after its pass 1
    (~26 at 4K on a whole MI355X: fewer and a pass-2 task waits holding its slot).  Frame
    k+1's tile row r waits for frame k's pass 2 of rows r-1..r+1, so consecutive frames trail
    each other by ~lag + 2 rows and the GOP's chain takes ~F (lag + 2) row-times, against
    F ntr / N row-times of work per rank: past N (lag + 2) > ntr the chain, not the CUs, sets
    the pace, hence lag <= ntr / N - 2 (4K: 20 at N = 3, 6 at N = 8).  Measured on one GPU with
    in-process ranks (tools/fpipe2p_probe.py, profiles/r03/fpipe2p_half.log): 3 ranks, 4K ROI +
    two-pass GOP, lag 26 / 12 / 5 -> 6.87 / 6.04 / 5.70 ms.  DESIGN.md section 6.1."""
    if world <= 2:
        return 0
    return max(3, ntr // world - 2)


class FramePipeRank:
    """One rank of a GOP whose frames are dealt round-robin over the ranks:
    rank g encodes one frame of every block of N consecutive frames (fpipe_plan: ranks 0..N-1
    in even blocks, 0, N-1, ..., 1 in odd ones; rank 0's frame 0 is the I-frame) with ONE
    persistent launch (so_encode_p_run_fpipe2); frame k's reference, frame k-1, arrives tile
    by tile from a ring neighbour into this rank's uncached landing plane of slot j (block j),
    and every tile of frame k is pushed on into the plane of the rank encoding frame k+1 (the
    next rank in even blocks, the previous one in odd blocks) as it completes.  Each rank encodes whole frames at full
    chip throughput while the frames of the other ranks run a couple of tile rows behind or
    ahead, so N ranks encode N frames at once; the only traffic is each reconstruction,
    once, over the xGMI link to the next rank."""

    def __init__(self, engine, world: int, rank: int, max_frames: int, stream=None, max_wg: int = 0,
                 p2lag=None):
        e = engine
        if world < 2:
            raise ValueError("the frame pipeline needs at least 2 ranks")
        if not e.pipelined_ok(1):
            raise ValueError("the frame pipeline covers bs 16 / sr 16 / full search / no FME / W % 128 == 0")
        self.eng, self.world, self.rank, self.max_frames = e, world, rank, max_frames
        self.stream, self.max_wg = stream, max_wg
        self.resident = _claim_slots(self, e, max_wg, e.vbs)
        lib = self.lib = _lib.load()
        self.tiles_x, self.ntr = e.w // 128, -(-e.nby // 2)
        self.ntiles = self.tiles_x * self.ntr
        self.p2lag = fpipe_p2lag(world, self.ntr) if p2lag is None else int(p2lag)
        self.nslots = fpipe_plan(world, rank, max_frames)["nslots"]
        self.stride = -(-(e.h * e.w + 256) // 256) * 256
        self._planes, self._flags = ctypes.c_void_p(), ctypes.c_void_p()
        _lib.check(lib.so_alloc_uncached(self.nslots * self.stride, ctypes.byref(self._planes)), "so_alloc_uncached")
        _lib.check(lib.so_alloc_uncached(self.nslots * self.ntiles * 4, ctypes.byref(self._flags)), "so_alloc_uncached")
        _lib.check(lib.so_memset_d8(self._planes, 0, self.nslots * self.stride, self._st()), "so_memset_d8")
        _lib.check(lib.so_memset_d8(self._flags, 0, self.nslots * self.ntiles * 4, self._st()), "so_memset_d8")
        self.epoch = 0
        self.peer = self.peer2 = None
        self._opened = []
        self._ws = torch.zeros(lib.so_p_run_workspace_elems(e.h, e.w), dtype=torch.int32, device=e.device)
        self.wait_health = runhealth.HealthLog()
        self._syms = None

    def _st(self):
        return self.stream.cuda_stream if self.stream is not None else _lib.stream_handle(self.eng.device)

    def frames_of(self, nframes: int) -> list:
        """Global indices of this rank's frames, in order (slot j <-> block j)."""
        return fpipe_plan(self.world, self.rank, nframes)["frames"]

    def info(self) -> dict:
        return {"planes": self._planes.value, "flags": self._flags.value, "rank": self.rank}

    def export(self) -> dict:
        hp, hf = (ctypes.c_uint8 * 64)(), (ctypes.c_uint8 * 64)()
        _lib.check(self.lib.so_ipc_export(self._planes, hp), "so_ipc_export")
        _lib.check(self.lib.so_ipc_export(self._flags, hf), "so_ipc_export")
        return {"planes_h": bytes(hp), "flags_h": bytes(hf), "rank": self.rank}

    def open(self, exported: dict) -> dict:
        out = {"rank": exported["rank"]}
        for k in ("planes", "flags"):
            p = ctypes.c_void_p()
            h = (ctypes.c_uint8 * 64).from_buffer_copy(exported[k + "_h"])
            _lib.check(self.lib.so_ipc_open(h, ctypes.byref(p)), "so_ipc_open")
            self._opened.append(p)
            out[k] = p.value
        return out

    def connect(self, nxt: dict, prv: dict | None = None) -> None:
        """nxt / prv: the next / previous rank's info() as mapped in this process (with two
        ranks they are the same rank; prv defaults to nxt then)."""
        if nxt["rank"] != (self.rank + 1) % self.world:
            raise ValueError("connect() takes the next rank")
        prv = nxt if prv is None and self.world == 2 else prv
        if prv is None or prv["rank"] != (self.rank - 1) % self.world:
            raise ValueError("connect() takes the previous rank too")
        self.peer = (nxt["planes"], nxt["flags"])
        self.peer2 = (prv["planes"], prv["flags"])

    def close(self) -> None:
        for p in self._opened:
            self.lib.so_ipc_close(p)
        self._opened = []
        for p in (self._planes, self._flags):
            if p.value:
                self.lib.so_free_device(p)
        self._planes, self._flags = ctypes.c_void_p(), ctypes.c_void_p()
        _release_slots(self)

    def prepare(self, nf: int, qp_row=None, two_pass: bool = False):
        """Allocate what encode() of an nf-frame GOP needs (this rank's symbol buffers, the QP
        maps, the row-QP constant) without launching anything; encode() calls it too.  Ranks
        sharing one GPU in one process (the tests) prepare every rank before any rank encodes,
        so that no host-side allocation runs while another rank's persistent grid is waiting.
        Returns (the symbols by global frame index, the row-QP tensor or None)."""
        e = self.eng
        mine = self.frames_of(nf)
        if self._syms is None or len(self._syms) != len(mine):
            self._syms = {k: e.new_symbols(0 if k == 0 else 1) for k in mine}
        if two_pass:
            for s in self._syms.values():
                if "qp_map" not in s.extra:
                    s.extra["qp_map"] = torch.empty(e.nb, dtype=torch.int32, device=e.device)
        return self._syms, (e.qp_row_tensor(qp_row) if qp_row is not None else None)

    def encode(self, frames: torch.Tensor, intra_dur: int, qp: int, qp_row=None, roi_dev=None,
               two_pass: bool = False, qp_clamp=(0, 12)) -> dict:
        """This rank's frames of the GOP {global index: FrameSymbols} (whole-frame symbols,
        local reconstructions).  Asynchronous on the rank's stream.

        Rate control (Y_Video_codec's RCFlag >= 1 without a P->I switch): qp_row = the per-row
        QP schedule (content-independent, Encoder.py:1599-1609, so every rank computes it);
        two_pass = RCFlag 3 (pass 1, the per-block QP map from the row's pass-1 tokens, pass 2;
        roi_dev: int32 [nb] ROI offsets, qp_clamp: the map's clamp) -- configs[4].  A rank owns
        whole frames, so the row-local statistics never cross ranks.  ROI without two-pass is
        not covered here (the stripes are)."""
        e, lib = self.eng, self.lib
        nf = frames.shape[0]
        if nf > self.max_frames or intra_dur < nf:
            raise ValueError("the frame pipeline runs one GOP of <= max_frames frames with its only I-frame first")
        if self.peer is None:
            raise RuntimeError("connect() first")
        if roi_dev is not None and not two_pass:
            raise ValueError("the frame pipeline covers ROI with two-pass RC only")
        if two_pass and e.vbs:
            raise ValueError("the frame pipeline's two-pass RC runs without VBSEnable")
        self.epoch += 1
        ep, st = self.epoch, self._st()
        mine = self.frames_of(nf)
        syms, qrd = self.prepare(nf, qp_row, two_pass)
        pplanes, pflags = self.peer
        ks = mine
        if self.rank == 0:
            s0 = syms[0]
            # the I-frame as encode_device's frame(): pass 1, the QP map, pass 2 (two-pass RC);
            # the engine launches on the current stream, i.e. the rank's
            with torch.cuda.stream(self.stream) if self.stream is not None else contextlib.nullcontext():
                e.encode_i(frames[0], qp, qp_row, out=s0, qp_row_dev=qrd)
                if two_pass:
                    qm = s0.extra["qp_map"]
                    e.qp_map(s0.tokens, qp, qrd, roi_dev, qm, qp_lo=qp_clamp[0], qp_hi=qp_clamp[1])
                    e.encode_i(frames[0], qp, qp_row, out=s0, qp_row_dev=qrd, qp_map_dev=qm)
            if nf > 1:   # frame 1 is rank 1's slot 0
                _lib.check(lib.so_frame_push(s0.recon.data_ptr(), e.h, e.w, pplanes, pflags, ep, st), "so_frame_push")
            ks = mine[1:]
        plan = fpipe_plan(self.world, self.rank, nf)
        if ks:
            n = len(ks)
            slot0 = plan["slot0"]
            arr = lambda xs: (ctypes.c_void_p * n)(*xs)  # noqa: E731
            ss = [syms[k] for k in ks]
            p2planes, p2flags = self.peer2
            outs = (arr([s.split.data_ptr() for s in ss]), arr([s.mv.data_ptr() for s in ss]),
                    arr([s.qtc.data_ptr() for s in ss]), arr([s.tokens.data_ptr() for s in ss]),
                    arr([s.mae_num.data_ptr() for s in ss]), arr([s.recon.data_ptr() for s in ss]),
                    arr([s.sse.data_ptr() for s in ss]))
            land = (self._planes.value, self._flags.value, slot0, pplanes, pflags, p2planes, p2flags,
                    (ctypes.c_int32 * n)(*plan["push"]), self.nslots, self.stride, ep, int(self.max_wg))
            curs = arr([frames[k].data_ptr() for k in ks])
            if two_pass:
                _lib.check(lib.so_encode_p_run_fpipe_2pass(
                    curs, n, e.h, e.w, e.bs, e.sr, int(qp), _lib.ptr(qrd), _lib.ptr(roi_dev), int(qp_clamp[0]),
                    int(qp_clamp[1]), *outs, arr([s.extra["qp_map"].data_ptr() for s in ss]), self._ws.data_ptr(),
                    *land, self.p2lag, st), "so_encode_p_run_fpipe_2pass")
            else:
                _lib.check(lib.so_encode_p_run_fpipe2(curs, n, e.h, e.w, e.bs, e.sr, int(qp), _lib.ptr(qrd), int(e.vbs),
                                                      e.lam, *outs, self._ws.data_ptr(), *land, st),
                           "so_encode_p_run_fpipe2")
            for s in ss:
                s.frame_type, s.qp_rd = 1, int(qp)
        for s in syms.values():
            s.qp_row = None if qp_row is None else list(qp_row)
        return syms

    def timed_out(self) -> bool:
        return runhealth.timed_out(self._ws)

    def check(self) -> None:
        """Raise (naming the first timed-out wait: landing slot, flags, GOP epoch) if a wait
        timed out since the last check; clear the counts."""
        runhealth.check(self._ws, self.wait_health, "p_run frame pipeline")


class FramePipelineGOPEncoder:
    """torch.distributed front end of FramePipeRank (one rank per GPU; the next rank's
    landing planes mapped by IPC, handles exchanged with all_gather_object)."""

    def __init__(self, engine, max_frames: int, group=None, max_wg: int = 0):
        import torch.distributed as dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.eng = engine
        self.r = FramePipeRank(engine, self.world, self.rank, max_frames, max_wg=max_wg)
        torch.cuda.synchronize(engine.device)
        alls = [None] * self.world
        dist.all_gather_object(alls, self.r.export(), group=group)
        nxt = self.r.open(alls[(self.rank + 1) % self.world])
        prv = nxt if self.world == 2 else self.r.open(alls[(self.rank - 1) % self.world])
        self.r.connect(nxt, prv)
        dist.barrier(group=group)

    def encode_local(self, frames, intra_dur: int, qp: int, **rc) -> dict:
        """This rank's launches only (no collective): {frame index: FrameSymbols}.  rc: the
        FramePipeRank.encode rate-control keywords."""
        return self.r.encode(frames, intra_dur, qp, **rc)

    def encode(self, frames, intra_dur: int, qp: int, syms: dict | None = None, reduce: bool = True, **rc) -> dict:
        """encode_local (unless its result is passed in) + one all_reduce of the per-frame SSE.

        reduce=False leaves "sse" None (sse() computes it later): no collective then joins
        the ranks between GOPs, so rank 0's next I-frame and the next GOP's first frames run
        while the other ranks finish this GOP's last frames -- the pipeline fill is paid once
        per stream, not once per GOP.  GOP k+1 may start on a rank as soon as its own GOP k
        launch is done: every landing slot it overwrites was last read by a frame that its
        own GOP k frames depend on.  That needs every rank to hold a frame
        after its first, i.e. nframes > world: with nframes <= world rank 0 has only the
        I-frame, and its next push into rank 1's slot 0 would race rank 1's read of it, so
        reduce=False is refused there (the all_reduce orders the GOPs instead)."""
        nf = frames.shape[0]
        if not reduce and nf <= self.world:
            raise ValueError(f"encode(reduce=False) needs more frames than ranks ({nf} <= {self.world}): "
                             "back-to-back GOPs would race on rank 1's first landing slot")
        syms = self.r.encode(frames, intra_dur, qp, **rc) if syms is None else syms
        return {"symbols": syms, "sse": self.sse(syms, nf) if reduce else None,
                "frame_type": [0 if k == 0 else 1 for k in range(nf)]}

    def sse(self, syms: dict, nframes: int) -> torch.Tensor:
        """The GOP's per-frame SSE on every rank (one all_reduce)."""
        import torch.distributed as dist
        sse = torch.zeros(nframes, dtype=torch.int64, device=self.eng.device)
        for k, s in syms.items():
            sse[k] = s.sse.sum(dtype=torch.int64)
        dist.all_reduce(sse, group=self.group)
        return sse

    def check(self) -> None:
        self.r.check()

    def digests(self, syms: dict, nframes: int) -> list:
        """Per-frame digests (digest.symbols_digest) of the whole GOP, on every rank."""
        import torch.distributed as dist
        from .digest import symbols_digest
        mine = {k: symbols_digest(s) for k, s in syms.items()}
        alls = [None] * self.world
        dist.all_gather_object(alls, mine, group=self.group)
        out = {}
        for d in alls:
            out.update(d)
        return [out[k] for k in range(nframes)]

    def close(self) -> None:
        self.r.close()
