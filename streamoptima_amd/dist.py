"""Stripe-sharded GOP encode across the GPUs of one node (BASELINE configs[3]).

Encoder.encode() (reference Encoder.py:1790-1898) is sequential over frames: P(i) needs
the reconstruction of frame i-1 (:1864-1867), so frames do not shard.
Blocks of one frame are independent given the reference, though:
  * ME reads only the previous reconstruction;
  * the residual and transform of a block read only that block;
  * intra mode 0 searches ORIGINAL pixels, and its reconstruction is row-local.

So rank r of N encodes the block rows [by0, by1) of every frame against the full previous
reconstruction, and then ONE collective per frame exchanges the stripes of the new
reconstruction. That collective is an in-place all_gather over RCCL/xGMI, or over gloo
in the CPU tests.

Layout for the exchange: every reconstruction plane is allocated with
`N * rows_per_rank * bs` rows, which may be more than H. Rank r's stripe then occupies
exactly chunk r of the flat buffer, and all_gather_into_tensor(flat, flat[chunk r]) fills
the plane in place with no copy. The padding rows past H are never read: the search
bounds are strict, and the kernels read at most 16 bytes of slack.

The symbols of a frame are the rank-order concatenation of the stripes, identical to a
1-GPU encode. The per-row RC QP schedule is content-independent (:1599-1609), so every
rank computes it locally. The RCFlag > 1 P->I switch (:1851-1856) needs the frame's total
residual size; that is one extra all_reduce of one int64 on the frames where it applies.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .engine import SLACK, FrameSymbols


def stripe_rows(nby: int, world: int, rank: int) -> tuple[int, int, int]:
    """Block-row range [by0, by1) of `rank` and the per-rank chunk height in block rows."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    rps = -(-nby // world)
    by0 = min(rank * rps, nby)
    by1 = min(by0 + rps, nby)
    return by0, by1, rps


class StripeGOPEncoder:
    """Encode GOPs with the block rows of every frame split across a process group.

    `engine` is a streamoptima_amd.engine.Engine (or anything with the same stripe
    methods: new_stripe_symbols, encode_p_rows, encode_i_rows, qp_row_tensor).
    """

    def __init__(self, engine, group=None):
        self.eng = engine
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.by0, self.by1, self.rps = stripe_rows(engine.nby, self.world, self.rank)
        self.chunk = self.rps * engine.bs * engine.w          # bytes of one rank's stripe

    # ---- planes ------------------------------------------------------------------------
    def new_plane(self, fill: int | None = None):
        """(flat buffer, [H, W] view) of a gather-ready reconstruction plane."""
        e = self.eng
        flat = torch.empty(self.world * self.chunk + SLACK, dtype=torch.uint8, device=e.device)
        if fill is not None:
            flat.fill_(fill)
        else:
            flat[self.world * self.chunk:].zero_()
        return flat, flat[: e.h * e.w].view(e.h, e.w)

    def exchange(self, flat: torch.Tensor) -> None:
        """All ranks' stripes of one reconstruction plane, in place."""
        if self.world == 1:
            return
        mine = flat[self.rank * self.chunk:(self.rank + 1) * self.chunk]
        dist.all_gather_into_tensor(flat[: self.world * self.chunk], mine, group=self.group)

    # ---- GOP -----------------------------------------------------------------------------
    def encode(self, frames: torch.Tensor, intra_dur: int, qp: int, nref: int = 1, qp_sched=None,
               rc_flag=None, intra_thresh=None, roi=None, qp_clamp=(0, 12)):
        """The encode() loop over frames [F, H, W] resident on this rank's device.

        rc_flag 3 = two-pass RC and `roi` (flat int32 per-block QP offsets) = ROI (build
        extensions, Encoder.py facade): a block row lies inside one stripe, so each rank
        builds the per-block QP map of its own rows from its own pass-1 tokens (so_qp_map);
        the map never crosses ranks.
        Returns per frame the stripe-local FrameSymbols (recon = the full, exchanged plane),
        the frame types, and the whole-frame SSE (int64 [F], summed over ranks).
        """
        e = self.eng
        nframes = frames.shape[0]
        _, init = self.new_plane(fill=128)
        refs = [init]
        qp_dev = e.qp_row_tensor(qp_sched) if qp_sched is not None else None
        two_pass = rc_flag is not None and rc_flag >= 3
        roi_dev = torch.as_tensor(roi, dtype=torch.int32).to(e.device) if roi is not None else None
        use_map = two_pass or roi_dev is not None
        lo, hi = qp_clamp

        def stripe(cur, intra, qp_rd, plane):
            sym = e.new_stripe_symbols(0 if intra else 1, self.by0, self.by1, plane)
            if self.by1 <= self.by0:            # a rank past the last block row idles
                if use_map:   # but joins the QP-map all_gather like every rank (gather_symbols)
                    sym.extra["qp_map"] = torch.zeros(e.nb, dtype=torch.int32, device=e.device)
                return sym
            qmap = torch.empty(e.nb, dtype=torch.int32, device=e.device) if use_map else None

            def run(qm, reuse=False):
                if intra:
                    e.encode_i_rows(cur, self.by0, self.by1, qp_rd, sym, qp_row_dev=qp_dev, qp_map_dev=qm)
                else:
                    e.encode_p_rows(cur, refs, self.by0, self.by1, qp_rd, sym, qp_row_dev=qp_dev, qp_map_dev=qm,
                                    reuse_me=reuse)
            if two_pass:
                run(None)
                e.qp_map(sym.tokens, qp_rd, qp_dev, roi_dev, qmap, self.by0, self.by1, lo, hi)
                run(qmap, reuse=not intra)
            elif roi_dev is not None:
                e.qp_map(None, qp_rd, qp_dev, roi_dev, qmap, self.by0, self.by1, lo, hi)
                run(qmap)
            else:
                run(None)
            if qmap is not None:
                sym.extra["qp_map"] = qmap      # valid on this rank's rows only
            return sym

        syms, ftypes = [], []
        for i in range(nframes):
            cur = frames[i]
            flat, plane = self.new_plane()
            if i % intra_dur == 0:
                sym = stripe(cur, True, qp, plane)
            else:
                sym = stripe(cur, False, qp, plane)
                if rc_flag is not None and rc_flag > 1 and (rc_flag == 2 or intra_thresh is not None):
                    total = sym.tokens.sum(dtype=torch.int64).reshape(1)
                    if self.world > 1:
                        dist.all_reduce(total, group=self.group)
                    if int(total.item()) > intra_thresh:
                        # Encoder.py:1851-1856: redo as intra with the last row's QP
                        sym = stripe(cur, True, qp_sched[-1], plane)
            sym.qp_row = list(qp_sched) if qp_sched is not None else None
            sym.extra["flat"] = flat
            self.exchange(flat)
            syms.append(sym)
            ftypes.append(sym.frame_type)
            if i < nframes - 1:
                if len(refs) >= nref:
                    refs.pop(0)
                refs.append(plane)
        # per-block / per-row SSE from the kernels; one reduction for the whole GOP
        sse = torch.stack([s.sse for s in syms]).sum(dim=1, dtype=torch.int64)
        if self.world > 1:
            dist.all_reduce(sse, group=self.group)
        return {"symbols": syms, "frame_type": ftypes, "sse": sse}

    # ---- symbols -------------------------------------------------------------------------
    def gather_symbols(self, sym: FrameSymbols) -> dict:
        """Whole-frame symbols (rank-order concatenation of the stripes) on every rank."""
        e = self.eng
        out = {}
        nbx = e.nbx
        for name in ("split", "mv", "qtc", "tokens", "mae_num"):
            t = getattr(sym, name)
            rec = tuple(t.shape[1:])
            pad = torch.zeros((self.rps * nbx,) + rec, dtype=t.dtype, device=t.device)
            pad[: t.shape[0]].copy_(t)
            if self.world > 1:
                # exchanged as raw bytes: every backend (gloo included) moves uint8
                full = torch.empty((self.world * self.rps * nbx,) + rec, dtype=t.dtype, device=t.device)
                dist.all_gather_into_tensor(full.view(-1).view(torch.uint8), pad.view(-1).view(torch.uint8),
                                            group=self.group)
            else:
                full = pad
            out[name] = full[: e.nby * nbx]
        qm = sym.extra.get("qp_map") if sym.extra else None
        if qm is not None:
            # ROI / two-pass RC: each rank's map is valid on its own block rows only; the
            # frame's map is their rank-order concatenation, like every other symbol
            pad = torch.zeros(self.rps * nbx, dtype=torch.int32, device=qm.device)
            nrow = max(self.by1 - self.by0, 0) * nbx
            pad[:nrow].copy_(qm[self.by0 * nbx:self.by0 * nbx + nrow])
            full = torch.empty(self.world * self.rps * nbx, dtype=torch.int32, device=qm.device)
            if self.world > 1:
                dist.all_gather_into_tensor(full.view(torch.uint8), pad.view(torch.uint8), group=self.group)
            else:
                full.copy_(pad)
            out["qp_map"] = full[: e.nby * nbx]
        out["recon"] = sym.recon
        out["frame_type"] = sym.frame_type
        return out
