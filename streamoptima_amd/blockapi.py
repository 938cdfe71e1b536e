"""The reference's per-block and per-frame public methods, dispatched to the GPU.

Y_Video_codec (Encoder.py) inherits these so a caller of the reference API (SURVEY.md
§8(b)) finds every method it calls with the same signature, arguments and return shapes:

  find_best_match(current_block, ref_frames, x, y, block_size, search_range)   Encoder.py:678
  inter_prediction(current_frame, ref_frames, block_size, search_range, ...)    :462
  intra_prediction(current_frame, mode, block_size, search_range)               :1238
  apply_2d_dct(input_block) / apply_2d_idct(transformed_coefficient_block)      :779 / :810
  reconstruct_block(predicted_block, residual_block, Q)                         :824
  reconstruct_frame(mvs, ref_frames, approximated_residual_blocks, Qp_per_row, bs) :831
  calculate_RD_cost(frame_type, split, mae, residuals, ...)                     :1133
  calculate_metrics(original_frame, modified_frame)                             :934
  frac_me_reference_frame(ref_frames, block_size)                               :388

Where the reference works on one block, the GPU works on a frame or a batch:
  * find_best_match runs the frame search kernel (so_me_full_search / so_me_search_ex) on a
    plane holding the block at (x, y) and returns that block's record;
  * apply_2d_dct / apply_2d_idct / calculate_RD_cost / reconstruct_block take one block or
    a stack [..., N, N] of blocks through so_block_xform in one launch;
  * inter_prediction / intra_prediction run the frame encode kernels for the motion vectors,
    split decisions and MAEs, and gather the (unquantised) residual blocks on the device.
There is no CPU path: without the HIP library every method raises (_lib.HipPathError).

FMEEnable: the reference hands inter_prediction / find_best_match the FRAC frames
(frac_me_reference_frame, (2H-1) x (2W-1)) and doubled coordinates / range
(complete_inter_flow, :1647-1651).  F[2i][2j] is the reference frame itself, and its
odd-column phase tells whether the row sums wrapped (uint8 list) or not (float start
frame), so the kernels' own FME path (phase planes from the reference frame) applies.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .engine import Engine, alloc_planes
from .package import frame_mvs, symbols_to_host


def _u8_plane(a, dev) -> torch.Tensor:
    a = np.asarray(a)
    if a.dtype != np.uint8:
        if not (np.all(a == np.round(a)) and a.min() >= 0 and a.max() <= 255):
            raise ValueError("frames must hold integer pixel values in [0, 255]")
        a = a.astype(np.uint8)
    p = alloc_planes(1, a.shape[0], a.shape[1], dev)[0]
    p.copy_(torch.from_numpy(np.ascontiguousarray(a)))
    return p


def _frac_to_ref(frac) -> tuple[np.ndarray, bool]:
    """(reference frame, wrap flag) of a frac frame F = frac_me_reference_frame([r])[0]."""
    F = np.asarray(frac)
    r = F[0::2, 0::2]
    if not (np.all(r == np.round(r)) and r.min() >= 0 and r.max() <= 255):
        raise ValueError("not a frac frame of a uint8 reference (frac_me_reference_frame)")
    ri = r.astype(np.int64)
    h = ri[:, :-1] + ri[:, 1:]
    odd = F[0::2, 1::2]
    if np.array_equal(odd, ((h & 255) + 1) >> 1):
        return ri.astype(np.uint8), True
    if np.array_equal(odd, (h + 1) >> 1):
        return ri.astype(np.uint8), False
    raise ValueError("not a frac frame of a uint8 reference (frac_me_reference_frame)")


class BlockAPI:
    """Mixin of Y_Video_codec: the per-block public methods of the reference on the GPU."""

    # ---- helpers ------------------------------------------------------------------------------
    def _block_engine(self, h, w, bs, sr, vbs=False, me_mode=0, fme=False) -> Engine:
        cache = self.__dict__.setdefault("_block_engines", {})
        key = (h, w, bs, sr, bool(vbs), int(me_mode), bool(fme))
        if key not in cache:
            cache[key] = Engine(h, w, bs, sr, vbs, self.lam if self.lam is not None else 0.0, self.device,
                                me_mode=me_mode, fme=fme)
        return cache[key]

    def _xform(self, blocks: np.ndarray, inverse: bool, qp: int = -1):
        """so_block_xform over a stack [n, N, N] -> (tc, q, tokens) numpy (q/tokens with qp >= 0)."""
        lib = _lib.load()
        a = np.ascontiguousarray(blocks, dtype=np.float64)
        n, N = a.shape[0], a.shape[-1]
        if a.shape[1:] != (N, N) or N not in (8, 16):
            raise ValueError(f"blocks must be [n, N, N] with N in (8, 16), got {a.shape}")
        dev = self.device
        src = torch.from_numpy(a).to(dev)
        tc = torch.empty((n, N, N), dtype=torch.int32, device=dev)
        q = torch.empty_like(tc) if qp >= 0 else None
        tok = torch.empty(n, dtype=torch.int32, device=dev) if qp >= 0 else None
        _lib.check(lib.so_block_xform(src.data_ptr(), n, N, int(inverse), int(qp), tc.data_ptr(), _lib.ptr(q),
                                      _lib.ptr(tok), _lib.stream_handle(dev)), "so_block_xform")
        return (tc.cpu().numpy(), None if q is None else q.cpu().numpy(), None if tok is None else tok.cpu().numpy())

    def _stack(self, x):
        a = np.asarray(x, dtype=np.float64)
        return a.reshape(-1, a.shape[-2], a.shape[-1]), a.shape

    # ---- transforms (Encoder.py:779-827) ----------------------------------------------------------
    def apply_2d_dct(self, input_block):
        """np.round(dct(dct(b, axis=0, 'ortho'), axis=1, 'ortho')).astype(int), any [..., N, N]."""
        a, shape = self._stack(input_block)
        return self._xform(a, False)[0].reshape(shape).astype(int)

    def apply_2d_idct(self, transformed_coefficient_block):
        """np.round(idct(idct(b, axis=0, 'ortho'), axis=1, 'ortho')).astype(int), any [..., N, N]."""
        a, shape = self._stack(transformed_coefficient_block)
        return self._xform(a, True)[0].reshape(shape).astype(int)

    def reconstruct_block(self, predicted_block, residual_block, Q):
        """(pred + apply_2d_idct(rescale_QTC(QTC, Q))).astype(uint8): mod-256 wrap (:824-827)."""
        deq = self.rescale_QTC(np.asarray(residual_block), np.asarray(Q))
        return (np.asarray(predicted_block) + self.apply_2d_idct(deq)).astype(np.uint8)

    def calculate_RD_cost(self, frame_type, split, mae, residuals, block_size=None, sub_block_size=None, lam=None):
        """lam * bits + mae with bits from the token count of quantize_TC(apply_2d_dct(res), Q)
        (Encoder.py:1133-1158); Q = the current QP's matrix (self.Q), Qm1 for the sub-blocks."""
        lam = self.lam if lam is None else lam
        if split == 0:
            blocks = np.asarray(residuals, dtype=np.float64)[None]
            tok = self._xform(blocks, False, self.Qp)[2]
            bit_rate = (8 if frame_type == 0 else 8 * 2) + 8 * int(tok[0])
        else:
            blocks = np.stack([np.asarray(r, dtype=np.float64) for r in residuals])
            tok = self._xform(blocks, False, self.Qpm1)[2]
            bit_rate = 8 * 4 if frame_type == 0 else 8 * 4 * 2
            for t in tok:
                bit_rate = bit_rate + 8 * int(t)
        return lam * bit_rate + mae

    # ---- metrics (Encoder.py:934-935) -----------------------------------------------------------
    def calculate_metrics(self, original_frame, modified_frame):
        """(PSNR with data_range 255, SSIM).  PSNR = 10 log10(255^2 / MSE) from the device SSE
        (so_sse_u8); SSIM is out of scope (skimage is absent): NaN."""
        a, b = np.asarray(original_frame), np.asarray(modified_frame)
        if a.shape != b.shape:
            raise ValueError(f"shapes differ: {a.shape} vs {b.shape}")
        n = a.size
        if all(x.dtype == np.uint8 or (np.all(x == np.round(x)) and x.min() >= 0 and x.max() <= 255) for x in (a, b)):
            lib = _lib.load()
            pa, pb = _u8_plane(a.reshape(a.shape[0], -1), self.device), _u8_plane(b.reshape(b.shape[0], -1), self.device)
            acc = torch.zeros(1, dtype=torch.int64, device=self.device)
            _lib.check(lib.so_sse_u8(pa.data_ptr(), pb.data_ptr(), n, acc.data_ptr(), _lib.stream_handle(self.device)),
                       "so_sse_u8")
            sse = float(acc.item())
        else:
            ta = torch.from_numpy(a.astype(np.float64)).to(self.device)
            tb = torch.from_numpy(b.astype(np.float64)).to(self.device)
            sse = float(((ta - tb) ** 2).sum().item())
        mse = sse / n
        psnr = float("inf") if mse == 0 else float(10 * np.log10((255 ** 2) / mse))
        return psnr, float("nan")

    # ---- FME frac frame (Encoder.py:388-403) ----------------------------------------------------
    def frac_me_reference_frame(self, ref_frames, block_size=None):
        """The (2H-1) x (2W-1) float64 half-pel frame of each reference, built on the GPU from
        the four phase planes (so_fme_planes).  np.copy(ref_frames) is uint8 -- and the row
        sums wrap mod 256 -- only when every reference is uint8."""
        lib = _lib.load()
        wrap = all(np.asarray(r).dtype == np.uint8 for r in ref_frames)
        out = []
        for r in ref_frames:
            p = _u8_plane(r, self.device)
            h, w = p.shape
            stride = lib.so_fme_plane_stride(h, w)
            ws = torch.zeros(4 * stride, dtype=torch.uint8, device=self.device)
            _lib.check(lib.so_fme_planes(p.data_ptr(), h, w, int(wrap), ws.data_ptr(), _lib.stream_handle(self.device)),
                       "so_fme_planes")
            P = [ws[k * stride:k * stride + h * w].view(h, w) for k in range(4)]
            F = torch.empty((2 * h - 1, 2 * w - 1), dtype=torch.float64, device=self.device)
            F[0::2, 0::2] = P[0]
            F[0::2, 1::2] = P[1][:, : w - 1]
            F[1::2, 0::2] = P[2][: h - 1]
            F[1::2, 1::2] = P[3][: h - 1, : w - 1]
            out.append(F.cpu().numpy())
        return out

    # ---- motion search (Encoder.py:678-717) ------------------------------------------------------
    def _refs_for_search(self, ref_frames):
        """(uint8 reference planes on the device, fme wrap flag); FMEEnable: from frac frames."""
        if self.FMEEnable:
            pairs = [_frac_to_ref(F) for F in ref_frames]
            return [_u8_plane(r, self.device) for r, _ in pairs], all(wp for _, wp in pairs)
        return [_u8_plane(r, self.device) for r in ref_frames], True

    def find_best_match(self, current_block, ref_frames, x, y, block_size=None, search_range=None):
        """((dx, dy, ref), mae) of one block, mae = SAD / bs^2 (inf with (0, 0, 0) when no
        candidate is valid).  With FMEEnable, (x, y) and search_range are the doubled values
        complete_inter_flow passes and the MV is in half-pel units."""
        bs = self.block_size if block_size is None else block_size
        sr = self.search_range if search_range is None else search_range
        refs, wrap = self._refs_for_search(ref_frames)
        h, w = refs[0].shape
        if self.FMEEnable:
            if x % 2 or y % 2 or sr % 2:
                raise ValueError("FMEEnable: x, y and search_range are the doubled (half-pel) values")
            x, y, sr = x // 2, y // 2, sr // 2
        if x % bs or y % bs:
            raise ValueError(f"block origin ({x}, {y}) is not on the {bs}-pixel grid")
        blk = np.asarray(current_block)
        plane = np.zeros((h, w), np.uint8)
        plane[y:y + bs, x:x + bs] = blk
        cur = _u8_plane(plane, self.device)
        lib = _lib.load()
        best = torch.empty(((h // bs) * (w // bs), 4), dtype=torch.int32, device=self.device)
        st = _lib.stream_handle(self.device)
        if self.FMEEnable:
            eng = self._block_engine(h, w, bs, sr, fme=True)
            ws = eng.fme_workspace(len(refs))
            rc = lib.so_me_search_ex(cur.data_ptr(), _lib.ref_array(refs), len(refs), h, w, bs, sr, _lib.ME_FULL, 1,
                                     int(wrap), ws.data_ptr(), best.data_ptr(), None, st)
        else:
            rc = lib.so_me_full_search(cur.data_ptr(), _lib.ref_array(refs), len(refs), h, w, bs, sr, best.data_ptr(),
                                       None, st)
        _lib.check(rc, "find_best_match")
        dx, dy, r, sad = (int(v) for v in best[(y // bs) * (w // bs) + x // bs].cpu().tolist())
        if sad < 0:
            return (0, 0, 0), float("inf")
        return (dx, dy, r), sad / (bs * bs)

    # ---- frame predictions (Encoder.py:462-585, 1238-1347) ----------------------------------------
    def inter_prediction(self, current_frame, ref_frames, block_size=None, search_range=None, nRefFrames=None,
                         fast_me=False, mvp=(0, 0, 0)):
        """(mvs, average_mae, residual_per_block) of the serial branch of inter_prediction:
        mvs [(0, (dx, dy, ref)) | (1, [4 x (dx, dy, ref)])], the unquantised residual blocks
        cur - prediction (float64), and the mean block MAE (vbs_mae for split-eligible blocks)."""
        bs = self.block_size if block_size is None else block_size
        sr = self.search_range if search_range is None else search_range
        if tuple(mvp) != (0, 0, 0):
            raise NotImplementedError("inter_prediction: a fast_me predictor other than (0, 0, 0) at the frame start")
        refs, wrap = self._refs_for_search(ref_frames)
        if self.FMEEnable:
            sr //= 2
        cur_np = np.asarray(current_frame)
        h, w = refs[0].shape
        if cur_np.shape != (h, w):
            raise ValueError(f"current frame {cur_np.shape} and references {(h, w)} differ")
        nref = len(refs) if nRefFrames is None or not fast_me else min(nRefFrames, len(refs))
        me_mode = _lib.ME_FULL if not fast_me else (_lib.ME_FAST_PAR if self.ParallelMode == 2 else _lib.ME_FAST)
        eng = self._block_engine(h, w, bs, sr, self.VBSEnable, me_mode, self.FMEEnable)
        cur = _u8_plane(cur_np, self.device)
        sym = eng.encode_p(cur, refs[:nref], self.Qp, fme_wrap=wrap)
        host = symbols_to_host(sym)
        mvs = frame_mvs(host, bs)
        avg = self._avg_mae(host["mae_num"], bs)
        res = self._inter_residuals(cur, refs[:nref], ref_frames, host, bs, wrap)
        return mvs, avg, res

    def _inter_residuals(self, cur, refs, ref_frames, host, bs, wrap):
        """calculate_inter_frame_residual (:432-460) of every chosen (sub-)block, gathered on
        the device: the strict-bound prediction, FME's stride-2 sample or 128 block, or
        handle_boundary_conditions' zero-filled overlap (:750-768)."""
        dev = self.device
        h, w = cur.shape
        nbx = w // bs
        if self.FMEEnable:
            planes = torch.stack([torch.from_numpy(np.asarray(F, dtype=np.float64)).to(dev) for F in ref_frames])
            step = 2
        else:
            planes = torch.stack([r.to(torch.float64) for r in refs])
            step = 1
        PH, PW = planes.shape[1:]
        curf = cur.to(torch.float64)
        split = host["split"].astype(bool)
        mv = torch.from_numpy(host["mv"].astype(np.int64)).to(dev)           # [nb, 4, 3]
        nb = split.size
        b = torch.arange(nb, device=dev)
        bx, by = (b % nbx) * bs, (b // nbx) * bs

        def gather(ox, oy, d, size):
            px = step * ox + d[:, 0]
            py = step * oy + d[:, 1]
            rf = d[:, 2]
            ar = torch.arange(size, device=dev)
            ok = (px >= 0) & (px < PW - size) & (py >= 0) & (py < PH - size)
            if step == 2:
                ok2 = (px + 2 * size >= 0) & (px + 2 * size < PW - size) & (py + 2 * size >= 0) & (py + 2 * size < PH - size)
            rows_s = py[:, None] + step * ar[None, :]
            cols_s = px[:, None] + step * ar[None, :]
            rows_1 = py[:, None] + ar[None, :]
            cols_1 = px[:, None] + ar[None, :]
            inside = ((rows_1 >= 0) & (rows_1 < PH))[:, :, None] & ((cols_1 >= 0) & (cols_1 < PW))[:, None, :]
            r1 = rows_1.clamp(0, PH - 1)
            c1 = cols_1.clamp(0, PW - 1)
            edge = torch.where(inside, planes[rf[:, None, None], r1[:, :, None], c1[:, None, :]], 0.0)
            rs = rows_s.clamp(0, PH - 1)
            cs = cols_s.clamp(0, PW - 1)
            direct = planes[rf[:, None, None], rs[:, :, None], cs[:, None, :]]
            if step == 2:
                direct = torch.where(ok2[:, None, None], direct, 128.0)
            pred = torch.where(ok[:, None, None], direct, edge)
            cb = curf[oy[:, None, None] + ar[None, :, None], ox[:, None, None] + ar[None, None, :]]
            return cb - pred

        full = gather(bx, by, mv[:, 0], bs).cpu().numpy()
        sb = bs // 2
        subs = None
        if split.any():
            subs = []
            for j in range(4):
                subs.append(gather(bx + (j & 1) * sb, by + (j >> 1) * sb, mv[:, j], sb).cpu().numpy())
        out = []
        for i in range(nb):
            out.append((1, [subs[j][i] for j in range(4)]) if split[i] else (0, full[i]))
        return out

    def intra_prediction(self, current_frame, mode=0, block_size=None, search_range=None):
        """(mvs, average_mae, residual_per_block, ref_frame) of intra_prediction, mode 0:
        mvs [(0, dx) | (1, [dx x 4])] with dx = -1 at x == 0, the unquantised residuals
        against the in-loop canvas (original pixels left of the block, 128 from its column
        on), and the canvas after the frame -- every block written back as pred + residual,
        i.e. the frame itself as float64 (the reference's canvas is 288 x 352; here the frame's
        size)."""
        if mode != 0:
            raise NotImplementedError("only intra mode 0 (horizontal) is built")
        bs = self.block_size if block_size is None else block_size
        sr = self.search_range if search_range is None else search_range
        cur_np = np.asarray(current_frame)
        h, w = cur_np.shape
        eng = self._block_engine(h, w, bs, sr, self.VBSEnable)
        cur = _u8_plane(cur_np, self.device)
        sym = eng.encode_i(cur, self.Qp)
        host = symbols_to_host(sym)
        mvs = frame_mvs(host, bs)
        avg = self._avg_mae(host["mae_num"], bs)
        dev = self.device
        curf = cur.to(torch.float64)
        nbx = w // bs
        split = host["split"].astype(bool)
        mv = torch.from_numpy(host["mv"].astype(np.int64)).to(dev)     # [nb, 4]
        b = torch.arange(split.size, device=dev)
        bx, by = (b % nbx) * bs, (b // nbx) * bs

        def gather(ox, oy, dx, size):
            ar = torch.arange(size, device=dev)
            cx = ox[:, None] + dx[:, None] + ar[None, :]                  # [nb, size]
            rows = oy[:, None] + ar[None, :]
            src = curf[rows[:, :, None], cx.clamp(0, w - 1)[:, None, :]]
            # x == 0 blocks predict from 128 (their mv -1 is a marker); a sub-block's dx of
            # -1 is a real offset
            left = (cx < bx[:, None])[:, None, :] & (bx[:, None, None] != 0)
            pred = torch.where(left, src, 128.0)
            cb = curf[rows[:, :, None], (ox[:, None] + ar[None, :])[:, None, :]]
            return cb - pred

        full = gather(bx, by, mv[:, 0], bs).cpu().numpy()
        sb = bs // 2
        subs = [gather(bx + (j & 1) * sb, by + (j >> 1) * sb, mv[:, j], sb).cpu().numpy() for j in range(4)] \
            if split.any() else None
        res = [(1, [subs[j][i] for j in range(4)]) if split[i] else (0, full[i]) for i in range(split.size)]
        return mvs, avg, res, cur_np.astype(np.float64)

    # ---- reconstruct_frame (Encoder.py:831-932) ------------------------------------------------------
    def reconstruct_frame(self, mvs, ref_frames, approximated_residual_blocks, Qp_per_row, block_size):
        """The P-frame reconstruction from the mvs / QTC lists (so_inter_recon_ex): per-row QP
        from Qp_per_row under rate control (the last row's QP stays set, like set_Qp), the
        current QP otherwise; FMEEnable predicts from the frac frames of ref_frames."""
        bs = block_size
        refs = [_u8_plane(r, self.device) for r in ref_frames]
        h, w = refs[0].shape
        nb = len(mvs)
        split = np.zeros(nb, np.uint8)
        mv = np.zeros((nb, 4, 3), np.int16)
        qtc = np.zeros((nb, bs * bs), np.int16)
        q4 = bs * bs // 4
        for i, (m, q) in enumerate(zip(mvs, approximated_residual_blocks)):
            if m[0] == 0:
                mv[i, 0] = m[1]
                qtc[i] = np.asarray(q[1]).reshape(-1)
            else:
                split[i] = 1
                for j in range(4):
                    mv[i, j] = m[1][j]
                    qtc[i, j * q4:(j + 1) * q4] = np.asarray(q[1][j]).reshape(-1)
        rc = self.RCFlag is not None and self.RCFlag > 0
        eng = self._block_engine(h, w, bs, self.search_range, False, 0, self.FMEEnable)
        dev = self.device
        t = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
        wrap = all(np.asarray(r).dtype == np.uint8 for r in ref_frames)
        out = eng.recon_inter(refs, t(split), t(mv), t(qtc), self.Qp, qp_row=list(Qp_per_row) if rc else None,
                              fme_wrap=wrap)
        if rc and len(Qp_per_row):
            self.set_Qp(Qp_per_row[-1])
        return out.cpu().numpy()

