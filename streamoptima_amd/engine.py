"""Device-resident frame engine: HBM buffers + launches of the gfx950 kernels.

Everything here stays on the GPU: frames, reconstructions, symbols (split / mv / qtc /
tokens / mae) and scratch are torch uint8/int16/int32 tensors allocated once and reused;
each frame is one or two C-ABI calls on the current stream with no host synchronisation.
The Python facade (Encoder.py / decoder.py) builds the reference's data structures from
these tensors only when asked.
"""
from __future__ import annotations

import collections
import contextlib
from dataclasses import dataclass, field

import ctypes
import os

import torch

from . import _lib, runhealth

SLACK = 64  # bytes readable past every plane (kernels read aligned words at row ends)
RUN_TIMEOUT_WORD = runhealth.TIMEOUT_WORD     # so_encode_p_run workspace (include/streamoptima.h)
RUN_FALLBACK_WORD = runhealth.FALLBACK_WORD   # blocks whose SEA search took the dense fallback


def alloc_planes(n: int, h: int, w: int, device, fill: int | None = None) -> torch.Tensor:
    """[n, h, w] uint8 planes laid out back to back with SLACK bytes after the last one."""
    flat = torch.empty(n * h * w + SLACK, dtype=torch.uint8, device=device)
    if fill is not None:
        flat.fill_(fill)
    else:
        flat[n * h * w:].zero_()
    return flat[: n * h * w].view(n, h, w)


@dataclass
class FrameSymbols:
    """Per-frame output of the encode path (canonical layout, include/streamoptima.h)."""
    frame_type: int            # 0 = intra, 1 = inter
    split: torch.Tensor        # uint8 [nb]
    mv: torch.Tensor           # int16 [nb, 4, 3] (inter) or [nb, 4] (intra)
    qtc: torch.Tensor          # int16 [nb, bs*bs]
    tokens: torch.Tensor       # int32 [nb]
    mae_num: torch.Tensor      # int32 [nb]  (block MAE * bs^2, -1 = inf)
    recon: torch.Tensor        # uint8 [h, w]
    sse: torch.Tensor | None = None   # int32 [max(nb, h)]: per-block (P) / per-row (I) SSE, zero-padded
    qp_rd: int = 0
    qp_row: list | None = None
    extra: dict = field(default_factory=dict)


class Engine:
    """Kernels for one frame geometry on one device."""

    def __init__(self, height: int, width: int, block_size: int = 16, search_range: int = 16,
                 vbs: bool = False, lam: float | None = None, device=None, me_mode: int = 0, fme: bool = False):
        if height % block_size or width % block_size:
            raise ValueError(f"frame {width}x{height} is not a multiple of block_size {block_size}")
        self.h, self.w, self.bs, self.sr = height, width, block_size, search_range
        self.vbs = bool(vbs)
        self.lam = float(lam) if lam is not None else 0.0
        if self.vbs and lam is None:
            raise ValueError("VBSEnable needs lam (calculate_RD_cost multiplies by it)")
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.type != "cuda":
            raise _lib.HipPathError("the encode path runs on a ROCm GPU only (no CPU fallback)")
        self.lib = _lib.load()
        self.nbx, self.nby = width // block_size, height // block_size
        self.nb = self.nbx * self.nby
        ps = self.lib.so_p_frame_scratch_elems(height, width, block_size, int(self.vbs))
        is_ = self.lib.so_i_frame_scratch_elems(height, width, block_size)
        self.scratch = torch.empty(max(ps, is_), dtype=torch.int32, device=self.device)
        # ME variant (include/streamoptima.h SO_ME_*): fast_me / FMEEnable
        self.me_mode = int(me_mode)
        self.fme = bool(fme)
        self._fme_ws = None
        self._consts: collections.OrderedDict = collections.OrderedDict()   # device_const_i32 (LRU)
        self._pinned_consts: set = set()                                    # ... held by captured graphs
        self._pin_depth = 0   # > 0 inside pinned_consts()
        self.wait_health = runhealth.HealthLog()   # non-fatal wait counts of the persistent runs

    MAX_CONSTS = 4096

    def device_const_i32(self, values) -> torch.Tensor:
        """A read-only int32 device copy of `values`, uploaded once per distinct content, so
        a GOP replayed from a captured HIP graph issues no host->device copy.

        The cache is LRU-bounded at MAX_CONSTS entries, except that an entry looked up while
        a HIP graph is being captured on this device, or inside `with engine.pinned_consts():`,
        is pinned: a graph holds its raw device pointer, so evicting it would make a later replay
        read freed memory.  A constant fetched BEFORE a capture and only used inside it must be
        fetched again inside the capture or under pinned_consts() (the facade looks its constants
        up on every call, so a captured encode re-fetches them).  Pinned entries are dropped only
        by release_consts(), which the owner of such a graph calls once the graph is gone."""
        host = torch.as_tensor(values, dtype=torch.int32).contiguous()
        key = (tuple(host.shape), host.numpy().tobytes())
        t = self._consts.get(key)
        if t is None:
            t = self._consts[key] = host.to(self.device)
            if len(self._consts) > self.MAX_CONSTS:   # evict the least recently used unpinned entry
                for k in self._consts:
                    if k not in self._pinned_consts and k != key:
                        del self._consts[k]
                        break
        else:
            self._consts.move_to_end(key)
        if self._pin_depth > 0 or (self.device.type == "cuda" and torch.cuda.is_current_stream_capturing()):
            self._pinned_consts.add(key)
        return t

    @contextlib.contextmanager
    def pinned_consts(self):
        """Every device constant looked up inside the block is pinned (never LRU-evicted): for
        constants fetched ahead of a graph capture that the graph will use."""
        self._pin_depth += 1
        try:
            yield self
        finally:
            self._pin_depth -= 1

    def release_consts(self) -> None:
        """Drop the cached device constants (ROI offsets, row-QP schedules), pinned ones too.
        Only safe when no captured HIP graph that used them will be replayed again."""
        self._consts.clear()
        self._pinned_consts.clear()

    def fme_workspace(self, nref: int) -> torch.Tensor:
        """Phase planes of the references' frac frames (rebuilt by every FME call)."""
        need = self.lib.so_fme_workspace_bytes(self.h, self.w, nref)
        if self._fme_ws is None or self._fme_ws.numel() < need:
            self._fme_ws = torch.zeros(need, dtype=torch.uint8, device=self.device)
        return self._fme_ws

    # ---- allocation ----------------------------------------------------------------------
    def new_symbols(self, frame_type: int) -> FrameSymbols:
        d, nb, bs = self.device, self.nb, self.bs
        mv_shape = (nb, 4, 3) if frame_type == 1 else (nb, 4)
        return FrameSymbols(frame_type=frame_type,
                            split=torch.empty(nb, dtype=torch.uint8, device=d),
                            mv=torch.empty(mv_shape, dtype=torch.int16, device=d),
                            qtc=torch.empty((nb, bs * bs), dtype=torch.int16, device=d),
                            tokens=torch.empty(nb, dtype=torch.int32, device=d),
                            mae_num=torch.empty(nb, dtype=torch.int32, device=d),
                            recon=alloc_planes(1, self.h, self.w, d)[0],
                            sse=torch.zeros(max(nb, self.h), dtype=torch.int32, device=d))

    def qp_row_tensor(self, qp_row) -> torch.Tensor | None:
        if qp_row is None:
            return None
        t = torch.as_tensor(list(qp_row), dtype=torch.int32)
        if t.numel() != self.nby:
            raise ValueError(f"qp_row needs {self.nby} entries, got {t.numel()}")
        return self.device_const_i32(t)

    def _check_plane(self, t: torch.Tensor, name: str):
        if t.dtype != torch.uint8 or t.device != self.device or tuple(t.shape) != (self.h, self.w):
            raise ValueError(f"{name} must be a uint8 {self.h}x{self.w} tensor on {self.device}")
        if not t.is_contiguous():
            raise ValueError(f"{name} must be contiguous")

    # ---- encode -------------------------------------------------------------------------
    def encode_p(self, cur: torch.Tensor, refs: list, qp_rd: int, qp_row=None,
                 out: FrameSymbols | None = None, qp_row_dev: torch.Tensor | None = None,
                 fme_wrap: bool = True, qp_map_dev: torch.Tensor | None = None,
                 reuse_me: bool = False, tokens_only: bool = False) -> FrameSymbols:
        """complete_inter_flow (Encoder.py:1644) for one frame; asynchronous.
        fme_wrap: see so_encode_p_rows_ex (False while refs hold the float64 start frame);
        qp_map_dev: per-block QP (ROI / two-pass RC); reuse_me: keep the ME records of the
        previous encode_p of the same frame (pass 2); tokens_only: pass 1 of two-pass RC (only
        the tokens and the ME records are guaranteed, SO_TOKENS_ONLY)."""
        return self.encode_p_rows(cur, refs, 0, self.nby, qp_rd, out or self.new_symbols(1),
                                  qp_row_dev if qp_row_dev is not None else self.qp_row_tensor(qp_row),
                                  fme_wrap=fme_wrap, qp_map_dev=qp_map_dev, reuse_me=reuse_me, qp_row=qp_row,
                                  tokens_only=tokens_only)

    def encode_i(self, cur: torch.Tensor, qp_rd: int, qp_row=None, out: FrameSymbols | None = None,
                 qp_row_dev: torch.Tensor | None = None, qp_map_dev: torch.Tensor | None = None) -> FrameSymbols:
        """complete_intra_flow (Encoder.py:1582), intra_mode 0, for one frame; asynchronous."""
        return self.encode_i_rows(cur, 0, self.nby, qp_rd, out or self.new_symbols(0),
                                  qp_row_dev if qp_row_dev is not None else self.qp_row_tensor(qp_row),
                                  qp_map_dev=qp_map_dev, qp_row=qp_row)

    def qp_map(self, tokens: torch.Tensor | None, qp_rd: int, qp_row_dev: torch.Tensor | None,
               roi_dev: torch.Tensor | None, out: torch.Tensor, by0: int = 0, by1: int | None = None,
               qp_lo: int = 0, qp_hi: int = 12) -> torch.Tensor:
        """so_qp_map: the per-block QP map of ROI / two-pass RC into `out` (int32 [nb])."""
        by1 = self.nby if by1 is None else by1
        rc = self.lib.so_qp_map(_lib.ptr(tokens), self.h, self.w, self.bs, int(by0), int(by1), int(qp_rd),
                                _lib.ptr(qp_row_dev), _lib.ptr(roi_dev), int(qp_lo), int(qp_hi), out.data_ptr(),
                                _lib.stream_handle(self.device))
        _lib.check(rc, "so_qp_map")
        return out

    # ---- stripes (multi-GPU sharding) --------------------------------------
    def new_stripe_symbols(self, frame_type: int, by0: int, by1: int, recon: torch.Tensor) -> FrameSymbols:
        """Stripe-local symbol buffers for block rows [by0, by1); `recon` is the full plane
        the stripe's rows are written into."""
        d, bs = self.device, self.bs
        nbs = self.nbx * (by1 - by0)
        mv_shape = (nbs, 4, 3) if frame_type == 1 else (nbs, 4)
        return FrameSymbols(frame_type=frame_type,
                            split=torch.empty(nbs, dtype=torch.uint8, device=d),
                            mv=torch.empty(mv_shape, dtype=torch.int16, device=d),
                            qtc=torch.empty((nbs, bs * bs), dtype=torch.int16, device=d),
                            tokens=torch.empty(nbs, dtype=torch.int32, device=d),
                            mae_num=torch.empty(nbs, dtype=torch.int32, device=d),
                            recon=recon,
                            sse=torch.zeros(max(nbs, (by1 - by0) * bs), dtype=torch.int32, device=d),
                            extra={"by0": by0, "by1": by1})

    def encode_p_rows(self, cur, refs, by0: int, by1: int, qp_rd: int, out: FrameSymbols,
                      qp_row_dev: torch.Tensor | None = None, fme_wrap: bool = True,
                      qp_map_dev: torch.Tensor | None = None, reuse_me: bool = False, qp_row=None,
                      tokens_only: bool = False) -> FrameSymbols:
        """so_encode_p_rows(_ex): block rows [by0, by1) of a P-frame; asynchronous."""
        self._check_plane(cur, "cur")
        for k, r in enumerate(refs):
            self._check_plane(r, f"refs[{k}]")
        if not 1 <= len(refs) <= _lib.MAX_REF:
            raise ValueError(f"nRefFrames must be in [1, {_lib.MAX_REF}]")
        st = _lib.stream_handle(self.device)
        if self.me_mode == _lib.ME_FULL and not self.fme and qp_map_dev is None and not reuse_me and not tokens_only:
            rc = self.lib.so_encode_p_rows(
                cur.data_ptr(), _lib.ref_array(refs), len(refs), self.h, self.w, self.bs, self.sr, int(by0), int(by1),
                int(qp_rd), _lib.ptr(qp_row_dev), int(self.vbs), self.lam, out.split.data_ptr(), out.mv.data_ptr(),
                out.qtc.data_ptr(), out.tokens.data_ptr(), out.mae_num.data_ptr(), out.recon.data_ptr(),
                _lib.ptr(out.sse), self.scratch.data_ptr(), st)
            _lib.check(rc, "so_encode_p_rows")
        else:
            ws = self.fme_workspace(len(refs)) if self.fme else None
            rc = self.lib.so_encode_p_rows_ex(
                cur.data_ptr(), _lib.ref_array(refs), len(refs), self.h, self.w, self.bs, self.sr, int(by0), int(by1),
                int(qp_rd), _lib.ptr(qp_row_dev), _lib.ptr(qp_map_dev), int(self.vbs), self.lam, self.me_mode,
                int(self.fme), int(bool(fme_wrap)), _lib.ptr(ws), (_lib.REUSE_ME if reuse_me else 0) | (_lib.TOKENS_ONLY if tokens_only else 0),
                out.split.data_ptr(), out.mv.data_ptr(), out.qtc.data_ptr(), out.tokens.data_ptr(),
                out.mae_num.data_ptr(), out.recon.data_ptr(), _lib.ptr(out.sse), self.scratch.data_ptr(), st)
            _lib.check(rc, "so_encode_p_rows_ex")
        out.frame_type, out.qp_rd = 1, int(qp_rd)
        out.qp_row = None if qp_row is None else list(qp_row)
        return out

    # ---- P-frame runs (one persistent launch) ----------------------------------------------
    def pipelined_ok(self, nref: int = 1, vbs_ok: bool = True) -> bool:
        """The configurations encode_p_run covers: the fused search + transform kernel
        (bs 16, sr 16, full search, no FME, one reference) on whole 128-byte rows; VBSEnable
        too unless vbs_ok is False (the two-pass RC run and the stripe hand-off)."""
        return (self.bs == 16 and self.sr == 16 and self.me_mode == _lib.ME_FULL and not self.fme
                and (vbs_ok or not self.vbs) and nref == 1 and self.w % 128 == 0)

    def encode_p_run(self, curs: list, ref0: torch.Tensor, qp_rd: int, outs: list, qp_row=None,
                     qp_row_dev: torch.Tensor | None = None) -> list:
        """so_encode_p_run: a run of consecutive P-frames (frame i predicts from frame i-1's
        reconstruction, ref0 for the first) as one persistent launch whose workgroups start
        a tile of frame i as soon as the rows of frame i-1 its window reads are done, so
        only the run's last frame has a launch tail.  Symbols identical to per-frame
        encode_p; asynchronous."""
        if not self.pipelined_ok():
            raise ValueError("encode_p_run covers bs 16 / sr 16 / full search / no FME / W % 128 == 0")
        n = len(curs)
        if n == 0:
            return []
        qrd = qp_row_dev if qp_row_dev is not None else self.qp_row_tensor(qp_row)
        for t, name in [(ref0, "ref0")] + [(c, "cur") for c in curs]:
            self._check_plane(t, name)
        if getattr(self, "_run_ws", None) is None:
            # the timeout count (RUN_TIMEOUT_WORD) is zeroed here once and then only by check_run
            self._run_ws = torch.zeros(self.lib.so_p_run_workspace_elems(self.h, self.w), dtype=torch.int32,
                                       device=self.device)

        def arr(ts):
            return (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts])
        with self._zero_skip_option():
            rc = self.lib.so_encode_p_run(
                arr(curs), n, ref0.data_ptr(), self.h, self.w, self.bs, self.sr, int(qp_rd), _lib.ptr(qrd),
                int(self.vbs), self.lam,
                arr([o.split for o in outs]), arr([o.mv for o in outs]), arr([o.qtc for o in outs]),
                arr([o.tokens for o in outs]), arr([o.mae_num for o in outs]), arr([o.recon for o in outs]),
                arr([o.sse for o in outs]), self._run_ws.data_ptr(), _lib.stream_handle(self.device))
        _lib.check(rc, "so_encode_p_run")
        self._last_run_outs = list(outs)
        for o in outs:
            o.frame_type, o.qp_rd = 1, int(qp_rd)
            o.qp_row = None if qp_row is None else list(qp_row)
        return outs

    def encode_p_run_2pass(self, curs: list, ref0: torch.Tensor, qp_rd: int, outs: list, qp_maps: list,
                           qp_row=None, qp_row_dev: torch.Tensor | None = None, roi_dev: torch.Tensor | None = None,
                           qp_lo: int = 0, qp_hi: int = 12) -> list:
        """so_encode_p_run_2pass: a run of P-frames with two-pass rate control (pass 1 at the
        row QP, per-block QPs from the row's pass-1 token statistics and the ROI, pass 2 at
        those QPs on pass 1's motion vectors) as ONE persistent launch.  qp_maps[i] (int32
        [nb]) receives frame i's QPs.  Symbols identical to encode_p + qp_map + encode_p
        (reuse_me) per frame; asynchronous."""
        if not self.pipelined_ok(vbs_ok=False):
            raise ValueError("encode_p_run_2pass covers bs 16 / sr 16 / full search / no VBS, FME / W % 128 == 0")
        n = len(curs)
        if n == 0:
            return []
        qrd = qp_row_dev if qp_row_dev is not None else self.qp_row_tensor(qp_row)
        for t, name in [(ref0, "ref0")] + [(c, "cur") for c in curs]:
            self._check_plane(t, name)
        for m in qp_maps:
            if m.dtype != torch.int32 or m.numel() != self.nb or m.device != self.device or not m.is_contiguous():
                raise ValueError(f"qp_maps entries must be contiguous int32 [{self.nb}] on {self.device}")
        if getattr(self, "_run_ws", None) is None:
            self._run_ws = torch.zeros(self.lib.so_p_run_workspace_elems(self.h, self.w), dtype=torch.int32,
                                       device=self.device)

        def arr(ts):
            return (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts])
        rc = self.lib.so_encode_p_run_2pass(
            arr(curs), n, ref0.data_ptr(), self.h, self.w, self.bs, self.sr, int(qp_rd), _lib.ptr(qrd),
            _lib.ptr(roi_dev), int(qp_lo), int(qp_hi),
            arr([o.split for o in outs]), arr([o.mv for o in outs]), arr([o.qtc for o in outs]),
            arr([o.tokens for o in outs]), arr([o.mae_num for o in outs]), arr([o.recon for o in outs]),
            arr([o.sse for o in outs]), arr(qp_maps), self._run_ws.data_ptr(), _lib.stream_handle(self.device))
        _lib.check(rc, "so_encode_p_run_2pass")
        for o, m in zip(outs, qp_maps):
            o.frame_type, o.qp_rd = 1, int(qp_rd)
            o.qp_row = None if qp_row is None else list(qp_row)
            o.extra["qp_map"] = m
        return outs

    def encode_p_runs(self, runs: list, qp_rd: int, qp_row=None, qp_row_dev: torch.Tensor | None = None) -> list:
        """so_encode_p_runs: several independent P-frame runs -- runs[r] = (curs, ref0, outs),
        frame i of a run predicting from frame i-1's reconstruction and frame 0 from ref0 --
        in ONE persistent launch, interleaved frame by frame (A1 B1 A2 B2 ...) so that a frame
        of every run is in flight at once.  Each run's symbols are identical to encode_p_run
        of that run alone; asynchronous."""
        if not self.pipelined_ok():
            raise ValueError("encode_p_runs covers bs 16 / sr 16 / full search / no FME / W % 128 == 0")
        qrd = qp_row_dev if qp_row_dev is not None else self.qp_row_tensor(qp_row)
        curs, refs, ref_frame, outs, last = [], [], [], [], {}
        for k in range(max((len(r[0]) for r in runs), default=0)):
            for r, (rc, r0, ro) in enumerate(runs):
                if k >= len(rc):
                    continue
                if len(rc) != len(ro):
                    raise ValueError("encode_p_runs: a run's curs and outs differ in length")
                for t, name in ((rc[k], "cur"),) + (((r0, "ref0"),) if k == 0 else ()):
                    self._check_plane(t, name)
                curs.append(rc[k])
                refs.append(r0 if k == 0 else None)
                ref_frame.append(-1 if k == 0 else last[r])
                last[r] = len(outs)
                outs.append(ro[k])
        n = len(curs)
        if n == 0:
            return []
        if getattr(self, "_run_ws", None) is None:
            self._run_ws = torch.zeros(self.lib.so_p_run_workspace_elems(self.h, self.w), dtype=torch.int32,
                                       device=self.device)

        def arr(ts):
            return (ctypes.c_void_p * n)(*[0 if t is None else t.data_ptr() for t in ts])
        with self._zero_skip_option():
            rc = self.lib.so_encode_p_runs(
                arr(curs), n, arr(refs), (ctypes.c_int32 * n)(*ref_frame), self.h, self.w, self.bs, self.sr,
                int(qp_rd), _lib.ptr(qrd), int(self.vbs), self.lam, arr([o.split for o in outs]),
                arr([o.mv for o in outs]), arr([o.qtc for o in outs]), arr([o.tokens for o in outs]),
                arr([o.mae_num for o in outs]), arr([o.recon for o in outs]), arr([o.sse for o in outs]),
                self._run_ws.data_ptr(), _lib.stream_handle(self.device))
        _lib.check(rc, "so_encode_p_runs")
        self._last_run_outs = list(outs)
        for o in outs:
            o.frame_type, o.qp_rd = 1, int(qp_rd)
            o.qp_row = None if qp_row is None else list(qp_row)
        return [r[2] for r in runs]

    def run_timed_out(self) -> bool:
        """True if a dependency wait of any encode_p_run since the last check_run timed out
        (never expected: the run's symbols would then be unreliable).  Synchronises."""
        return runhealth.timed_out(getattr(self, "_run_ws", None))

    def _zero_skip_option(self):
        """SO_OPT_RUN_ZERO_SKIP set around a launch when this engine chose the zero-skip kernel
        (left alone otherwise: the option's default is off)."""
        return _lib.option(_lib.OPT_RUN_ZERO_SKIP, 1) if self.zero_skip else contextlib.nullcontext()

    # the plain run's kernel choice by content (SO_OPT_RUN_ZERO_SKIP): the instantiation that
    # skips the IDCT of all-zero waves when at least this share of the last run's blocks
    # quantised to zero (flat content; exact either way)
    ZERO_SKIP_SHARE = float(os.environ.get("SO_ZERO_SKIP_SHARE", "0.5"))   # A/B: the share that selects it
    zero_skip = False

    def check_run(self, defer_stats: bool = False) -> None:
        """Raise if any encode_p_run since the last check timed out -- naming the first such
        wait from the workspace's diagnostic record (runhealth.describe) -- then clear the
        count; the non-fatal wait counts go to self.wait_health.  Encoder.encode() /
        encode_device(check=True) and bench.py call it once per GOP.  It also picks the
        plain run's kernel for the next runs from the last run's share of all-zero blocks
        (tokens == 1), read in the same synchronised check -- or, with defer_stats, counted
        on the stream into page-locked memory and read at the next check (one GOP later; the
        host-stream region, hoststream.py, does not wait for it)."""
        runhealth.check(getattr(self, "_run_ws", None), self.wait_health, "p_run_kernel")
        pend = getattr(self, "_zero_pending", None)
        if pend is not None:
            self._zero_pending = None
            ev, host, blocks = pend
            ev.synchronize()
            self.zero_skip = int(host[0]) >= self.ZERO_SKIP_SHARE * blocks
        outs = getattr(self, "_last_run_outs", None)
        if outs and not self.vbs:
            self._last_run_outs = None
            zero = torch.stack([(o.tokens == 1).sum() for o in outs]).sum()
            if defer_stats:
                if getattr(self, "_zero_host", None) is None:
                    self._zero_host = torch.empty(1, dtype=torch.int64, pin_memory=True)
                self._zero_host.copy_(zero.view(1), non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
                self._zero_pending = (ev, self._zero_host, self.nb * len(outs))
            else:
                self.zero_skip = zero.item() >= self.ZERO_SKIP_SHARE * self.nb * len(outs)

    def take_sad_ops(self) -> int:
        """SAD byte operations the persistent runs' searches executed since the last call
        (SO_P_RUN_SAD_OPS_WORD); clears the count.  Synchronises."""
        ws = getattr(self, "_run_ws", None)
        return 0 if ws is None else runhealth.take_u64(ws, runhealth.SAD_OPS_WORD)

    def take_fallback_count(self) -> int:
        """Blocks of the persistent runs since the last call whose exact SEA search took the
        dense fallback (SO_P_RUN_FALLBACK_WORD); clears the count.  Synchronises."""
        ws = getattr(self, "_run_ws", None)
        if ws is None:
            return 0
        n = int(ws[RUN_FALLBACK_WORD].item())
        ws[RUN_FALLBACK_WORD].zero_()
        return n

    def encode_i_rows(self, cur, by0: int, by1: int, qp_rd: int, out: FrameSymbols,
                      qp_row_dev: torch.Tensor | None = None, qp_map_dev: torch.Tensor | None = None,
                      qp_row=None) -> FrameSymbols:
        """so_encode_i_rows_ex: block rows [by0, by1) of an I-frame; asynchronous."""
        self._check_plane(cur, "cur")
        rc = self.lib.so_encode_i_rows_ex(
            cur.data_ptr(), self.h, self.w, self.bs, self.sr, int(by0), int(by1), int(qp_rd), _lib.ptr(qp_row_dev),
            _lib.ptr(qp_map_dev), int(self.vbs), self.lam, out.split.data_ptr(), out.mv.data_ptr(),
            out.qtc.data_ptr(), out.tokens.data_ptr(), out.mae_num.data_ptr(), out.recon.data_ptr(),
            _lib.ptr(out.sse), self.scratch.data_ptr(), _lib.stream_handle(self.device))
        _lib.check(rc, "so_encode_i_rows_ex")
        out.frame_type, out.qp_rd = 0, int(qp_rd)
        out.qp_row = None if qp_row is None else list(qp_row)
        return out

    # ---- decode ---------------------------------------------------------------------------
    def recon_inter(self, refs: list, split, mv, qtc, qp: int, qp_row=None, out=None,
                    fme_wrap: bool = True, qp_map_dev: torch.Tensor | None = None) -> torch.Tensor:
        out = out if out is not None else alloc_planes(1, self.h, self.w, self.device)[0]
        qr = self.qp_row_tensor(qp_row)
        ws = self.fme_workspace(len(refs)) if self.fme else None
        rc = self.lib.so_inter_recon_ex(_lib.ref_array(refs), len(refs), self.h, self.w, self.bs, int(qp),
                                        _lib.ptr(qr), _lib.ptr(qp_map_dev), int(self.fme), int(bool(fme_wrap)),
                                        _lib.ptr(ws), split.data_ptr(), mv.data_ptr(), qtc.data_ptr(), out.data_ptr(),
                                        _lib.stream_handle(self.device))
        _lib.check(rc, "so_inter_recon_ex")
        return out

    def recon_intra(self, split, mv, qtc, qp: int, qp_row=None, out=None,
                    qp_map_dev: torch.Tensor | None = None) -> torch.Tensor:
        out = out if out is not None else alloc_planes(1, self.h, self.w, self.device)[0]
        qr = self.qp_row_tensor(qp_row)
        rc = self.lib.so_intra_recon_ex(self.h, self.w, self.bs, int(qp), _lib.ptr(qr), _lib.ptr(qp_map_dev),
                                        split.data_ptr(), mv.data_ptr(), qtc.data_ptr(), out.data_ptr(),
                                        self.scratch.data_ptr(), _lib.stream_handle(self.device))
        _lib.check(rc, "so_intra_recon_ex")
        return out

    # ---- packed symbol stream (so_pack_frames) --------------------------------------------
    def pack_bound(self, nb: int | None = None) -> int:
        return int(self.lib.so_pack_bound(int(self.nb if nb is None else nb), self.bs))

    def pack_symbols(self, syms: list, offs: torch.Tensor | None = None, out: torch.Tensor | None = None,
                     totals_ptr: int | None = None):
        """Each frame's symbols as one packed byte stream on the device (include/streamoptima.h
        so_pack_frames); asynchronous.  Returns (offs int32 [n, nb + 1], out uint8 [n, cap]):
        frame i's stream is out[i, :offs[i, nb]], block b starts at offs[i, b]
        (bitstream.unpack_frame decodes it).  The default capacity never overflows.
        totals_ptr: a device address of n uint32 (hostmem.device_ptr of a page-locked host
        array) that also receives offs[i, nb] (so_pack_frames_ex)."""
        n = len(syms)
        if n == 0:
            raise ValueError("pack_symbols: no frames")
        nb = syms[0].split.numel()
        if any(s.split.numel() != nb for s in syms):
            raise ValueError("pack_symbols: frames with different block counts")
        cap = self.pack_bound(nb) if out is None else out.shape[1]
        offs = torch.empty((n, nb + 1), dtype=torch.int32, device=self.device) if offs is None else offs
        out = torch.empty((n, cap), dtype=torch.uint8, device=self.device) if out is None else out
        if offs.shape != (n, nb + 1) or offs.dtype != torch.int32 or out.shape[0] != n or out.dtype != torch.uint8:
            raise ValueError("pack_symbols: offs must be int32 [n, nb + 1] and out uint8 [n, cap]")

        def arr(ts):
            return (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts])
        types = (ctypes.c_int32 * n)(*[int(s.frame_type) for s in syms])
        rc = self.lib.so_pack_frames_ex(n, types, arr([s.split for s in syms]), arr([s.mv for s in syms]),
                                        arr([s.qtc for s in syms]), nb, self.bs, arr(list(offs)), arr(list(out)),
                                        int(cap), totals_ptr, _lib.stream_handle(self.device))
        _lib.check(rc, "so_pack_frames")
        return offs, out

    def unpack_symbols(self, frame_types: list, packed: list, offs: list) -> list:
        """so_unpack_frames: packed streams (device uint8) + their block offsets (device int32
        [nb + 1], as pack_symbols wrote them) -> FrameSymbols with split / mv / qtc (no recon,
        tokens or metrics).  Raises ValueError on a malformed stream (synchronises once)."""
        n = len(packed)
        syms = [self.new_symbols(int(t)) for t in frame_types]
        err = torch.zeros(1, dtype=torch.int32, device=self.device)

        def arr(ts):
            return (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts])
        types = (ctypes.c_int32 * n)(*[int(t) for t in frame_types])
        rc = self.lib.so_unpack_frames(n, types, arr(packed), arr(offs), self.nb, self.bs, arr([s.split for s in syms]),
                                       arr([s.mv for s in syms]), arr([s.qtc for s in syms]), err.data_ptr(),
                                       _lib.stream_handle(self.device))
        _lib.check(rc, "so_unpack_frames")
        bad = int(err.item())
        if bad:
            raise ValueError(f"so_unpack_frames: malformed packed stream at block {bad - 1}")
        return syms

    # ---- metrics ---------------------------------------------------------------------------
    def sum_rows(self, rows: list, out: torch.Tensor | None = None) -> torch.Tensor:
        """int64 [n]: the sum of each int32 tensor in `rows` (equal lengths), one launch."""
        n = len(rows)
        length = rows[0].numel() if n else 0
        if any(r.numel() != length or r.dtype != torch.int32 or not r.is_contiguous() for r in rows):
            raise ValueError("sum_rows: contiguous int32 tensors of one length")
        out = torch.empty(n, dtype=torch.int64, device=self.device) if out is None else out
        ptrs = (ctypes.c_void_p * max(n, 1))(*[r.data_ptr() for r in rows])
        rc = self.lib.so_sum_i32_rows(ptrs, n, length, out.data_ptr(), _lib.stream_handle(self.device))
        _lib.check(rc, "so_sum_i32_rows")
        return out

    def sse_into(self, a: torch.Tensor, b: torch.Tensor, acc: torch.Tensor) -> None:
        """acc (uint64 view of an int64 device scalar) += sum((a-b)^2)."""
        rc = self.lib.so_sse_u8(a.data_ptr(), b.data_ptr(), a.numel(), acc.data_ptr(),
                                _lib.stream_handle(self.device))
        _lib.check(rc, "so_sse_u8")
