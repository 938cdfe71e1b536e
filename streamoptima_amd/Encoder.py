"""Drop-in `Y_Video_codec` (the reference's Encoder.py surface) on the MI355X path.

Same constructor, attributes and public methods as Suyashagarw/StreamOptima's
Encoder.Y_Video_codec (Encoder.py:17-1898).  The per-frame work runs in the gfx950
library (libstreamoptima_hip.so) on HBM-resident frames; this module keeps the host-side
control flow of the reference: GOP cadence, reference window, QP reset per frame, the
per-row rate-control schedule, the RCFlag > 1 P->I switch, PSNR, the closed-loop decode,
the `encoded_package` dict and the text bitstream.

Deliberate, documented deviations ("Boundary"):
  * frames whose height/width are not multiples of block_size are padded with 128
    (pad_hw) and encoded at the padded size; the reference crashes there (Encoder.py:930);
  * the intra canvas is frame-sized (the reference hard-codes 288x352, Encoder.py:1248);
  * intra_mode 1 and ParallelMode 1/3 raise NotImplementedError (mode 1 changes semantics,
    mode 3 is broken upstream).  ParallelMode 2 is accepted: it is serial-identical in the
    reference except under fast_me, where every block's predictor is (0,0,0) with one
    reference (inter_prediction_parallel, Encoder.py:587-676) -- SO_ME_FAST_PAR; fast_me +
    VBSEnable under ParallelMode 2 raises NameError in the reference and ValueError here.
  * fast_me and FMEEnable run on the GPU (so_encode_p_rows_ex, so_fastme.hip / the FME
    phase-plane search in so_me.hip).
"""
from __future__ import annotations

import math
import os
import time

import numpy as np
import torch

from . import decoder as _decoder_mod
from .engine import Engine, FrameSymbols, alloc_planes
from .blockapi import BlockAPI
from .bitstream import (differential_encoder_frame as _diff_enc, entropy_encoder_block as _ent_blk,
                        entropy_encoder_frame as _ent_frame)
from .package import LazyPackage, frame_mvs, frame_residuals, symbols_to_host


def _psnr_from_sse(sse: int, n: int) -> float:
    # skimage.metrics.peak_signal_noise_ratio(data_range=255): 10*log10(255^2 / mean((a-b)^2))
    if sse == 0:
        return float("inf")
    mse = float(sse) / float(n)
    return float(10 * np.log10((255 ** 2) / mse))


class Y_Video_codec(BlockAPI):
    """See Encoder.py:24 of the reference for the argument meanings.  The per-block public
    methods (find_best_match, inter_prediction, apply_2d_dct, ...) come from BlockAPI."""

    def __init__(self, h_pixels, w_pixels, frames, block_size, search_range, Qp, intra_dur, intra_mode,
                 lam=None, VBSEnable=False, nRefFrames=1, yuv_file=None, y_only_frame_arr=None,
                 fast_me=False, FMEEnable=False, RCFlag=None, targetBR=None, frame_rate=30,
                 qp_rate_tables=None, intra_thresh=None, ParallelMode=0, device=None, roi=None, qp_clamp=(0, 12)):
        if fast_me and ParallelMode == 2 and VBSEnable:
            raise ValueError("fast_me + VBSEnable under ParallelMode 2: the reference raises NameError on "
                             "`mvp` (inter_prediction_parallel, Encoder.py:609)")
        if intra_mode not in (0,):
            raise NotImplementedError("only intra_mode 0 (horizontal) is built")
        if ParallelMode not in (0, 2):
            raise NotImplementedError("ParallelMode 1 changes semantics and 3 is broken in the reference")
        if RCFlag is not None and RCFlag > 3:
            raise ValueError(f"RCFlag {RCFlag}: 0-2 are the reference's, 3 is two-pass RC (build extension)")
        self.h_pixels = h_pixels
        self.w_pixels = w_pixels
        self.frames = frames
        self.block_size = block_size
        self.num_blocks_per_row = w_pixels / block_size
        self.sub_block_size = block_size // 2
        self.search_range = search_range
        self.Qp = Qp
        self.const_init_Qp = Qp
        self.intra_dur = intra_dur
        self.intra_mode = intra_mode
        self.nRefFrames = nRefFrames
        self.fast_me = fast_me
        self.FMEEnable = FMEEnable
        self.VBSEnable = VBSEnable
        self.lam = lam
        self.RCFlag = RCFlag
        self.target_bitrate = None
        self.bitrate_per_row = None
        self.frame_rate = frame_rate
        self.qr_rate_tables = qp_rate_tables
        self.intra_thresh = intra_thresh
        self.ParallelMode = ParallelMode
        self.encoded_package = None
        self.encoded_package_f = False
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.recon_yuv_path = "yuv/y_only_reconstructed.yuv"
        self.inter0, self.intra0, self.inter1, self.intra1 = [], [], [], []
        self.inter2, self.intra2, self.inter3, self.intra3 = [], [], [], []
        self.Q = self.generate_Q_matrix(block_size, Qp)
        self.Qpm1 = Qp - 1 if Qp > 0 else Qp
        self.Qm1 = self.generate_Q_matrix(self.sub_block_size, self.Qpm1)
        if targetBR is not None:
            self.set_target_bitrate(targetBR)
        self.decoder = _decoder_mod.decoder(intra_mode, intra_dur, block_size, frames, h_pixels, w_pixels, Qp,
                                            nRefFrames, FMEEnable, lam, VBSEnable, False, RCFlag, targetBR,
                                            frame_rate, qp_rate_tables, ParallelMode=ParallelMode,
                                            device=self.device)
        if yuv_file is not None:
            self.y_only_f_arr = self.read_yuv(yuv_file, h_pixels, w_pixels, frames)
        else:
            self.y_only_f_arr = y_only_frame_arr
        # build extension (BASELINE configs[4], DESIGN.md "ROI and two-pass rate control"):
        # roi = per-block QP offsets ([H/bs, W/bs] array) or rectangles (x0, y0, x1, y1, offset)
        # in pixels -- a block takes the offset of the last rectangle holding its centre;
        # RCFlag 3 = two-pass RC (pass-1 token counts -> per-block QP map, so_qp_map)
        self.roi = roi
        self.qp_clamp = tuple(qp_clamp)
        self._engine = None
        self._symbols = None

    def roi_block_offsets(self):
        """ROI as int32 [nb] per-block QP offsets (raster order), or None."""
        from .workloads import roi_offsets
        return roi_offsets(self.roi, self.h_pixels, self.w_pixels, self.block_size)

    # ---- host helpers with the reference's semantics ---------------------------------------
    def set_target_bitrate(self, targetBR):
        """Encoder.py:78-88 ('<n> bps|kbps|mbps'; kbps = 1024, mbps = 1048576)."""
        tokens = targetBR.split(" ")
        num = int(tokens[0])
        if tokens[1] == "kbps":
            self.target_bitrate = num * 1024
        elif tokens[1] == "mbps":
            self.target_bitrate = num * 1048576
        else:
            self.target_bitrate = num
        self.bitrate_per_row = (self.target_bitrate // self.frame_rate) / (self.h_pixels / self.block_size)

    @staticmethod
    def read_yuv(raw_yuv_420_f, height, width, frames):
        """Y planes of a 4:2:0 file (Encoder.py:110-126)."""
        size_y = width * height
        size_uv = size_y // 4
        out = np.empty((frames, height, width), dtype=np.uint8)
        with open(raw_yuv_420_f, "rb") as f:
            for i in range(frames):
                out[i] = np.frombuffer(f.read(size_y), dtype=np.uint8).reshape(height, width)
                f.read(size_uv * 2)
        return out

    def pad_hw(self, array, i, pad_with=None):
        """Encoder.py:140-155: pad to a multiple of i (float64, like the reference)."""
        r_req = math.ceil(self.h_pixels / i)
        c_req = math.ceil(self.w_pixels / i)
        result = np.zeros((r_req * i, c_req * i)) + (0 if pad_with is None else pad_with)
        arr_r, arr_c = array.shape
        result[0:arr_r, 0:arr_c] = array
        return result

    @staticmethod
    def generate_Q_matrix(i, QP):
        """Encoder.py:938-945."""
        x = np.arange(i)[:, None] + np.arange(i)[None, :]
        return np.where(x < i - 1, 2 ** QP, np.where(x == i - 1, 2 ** (QP + 1), 2 ** (QP + 2))).astype(int)

    def set_Qp(self, Qp):
        """Encoder.py:948-959."""
        self.Qp = Qp
        self.Q = self.generate_Q_matrix(self.block_size, Qp)
        self.Qpm1 = Qp - 1 if Qp > 0 else Qp
        self.Qm1 = self.generate_Q_matrix(self.sub_block_size, self.Qpm1)

    def get_appropriate_Qp_value(self, frame_type, row_bit_budget):
        """Encoder.py:1576-1580: first QP whose table entry is below the budget (else None)."""
        for Qp, bitrate in enumerate(self.qr_rate_tables[frame_type]):
            if bitrate < row_bit_budget:
                return Qp, bitrate
        return None

    def row_qp_schedule(self, n_rows):
        """The per-row QP loop of complete_inter_flow / complete_intra_flow
        (Encoder.py:1599-1609, 1668-1678).  Content independent; both frame types use
        table 0 exactly as the reference does (:1671, :1676)."""
        qps = []
        budget, spent = self.bitrate_per_row, 0
        for r in range(n_rows):
            if r == 0:
                budget = self.bitrate_per_row
            else:
                budget = self.bitrate_per_row + (budget - spent)
            got = self.get_appropriate_Qp_value(0, budget)
            if got is None:
                raise TypeError("cannot unpack non-iterable NoneType object "
                                f"(no QP in qp_rate_tables[0] fits the row budget {budget})")
            q, spent = got
            qps.append(q)
        return qps

    # ---- per-block helpers kept for API compatibility (host bitstream logic) -------------
    def entropy_encoder_block(self, residual_block, block_size):
        return _ent_blk(residual_block, block_size)

    def quantize_TC(self, TC, Q):
        return np.round(TC / Q).astype(int)

    def rescale_QTC(self, QTC, Q):
        return QTC * Q

    def differential_encoder_frame(self, frame_type, mv_for_frame, Qp_for_frame):
        return _diff_enc(frame_type, mv_for_frame, Qp_for_frame, self.RCFlag, self.num_blocks_per_row)

    def entropy_encoder_frame(self, frame_residuals, block_size=None):
        return _ent_frame(frame_residuals, block_size or self.block_size)

    # ---- device plumbing -----------------------------------------------------------------
    def _geometry(self):
        bs = self.block_size
        hp = math.ceil(self.h_pixels / bs) * bs
        wp = math.ceil(self.w_pixels / bs) * bs
        return hp, wp

    def engine(self) -> Engine:
        hp, wp = self._geometry()
        if self._engine is None or (self._engine.h, self._engine.w) != (hp, wp):
            self._engine = Engine(hp, wp, self.block_size, self.search_range, self.VBSEnable, self.lam,
                                  self.device, me_mode=self._me_mode(), fme=bool(self.FMEEnable))
        return self._engine

    def _me_mode(self) -> int:
        """SO_ME_* of this configuration (include/streamoptima.h)."""
        from . import _lib
        if not self.fast_me:
            return _lib.ME_FULL
        return _lib.ME_FAST_PAR if self.ParallelMode == 2 else _lib.ME_FAST

    def _upload_padded(self, arr) -> torch.Tensor:
        """host frames -> [F, Hp, Wp] uint8 planes in HBM (pad_hw with 128)."""
        a = np.asarray(arr)
        if a.ndim == 2:
            a = a[None]
        hp, wp = self._geometry()
        f, h, w = a.shape
        planes = alloc_planes(f, hp, wp, self.device)
        src = torch.from_numpy(np.ascontiguousarray(a.astype(np.uint8, copy=False)))
        if (h, w) != (hp, wp):
            planes.fill_(128)
            planes[:, :h, :w].copy_(src, non_blocking=False)
        else:
            planes.copy_(src)
        return planes

    def _rc_on(self):
        return self.RCFlag is not None and self.RCFlag > 0

    # ---- frame flows (reference signatures) ---------------------------------------------
    def complete_inter_flow(self, current_padded_frame, ref_frames, block_size, search_range,
                            generate_row_wise_stats=True):
        """Encoder.py:1644-1709 on the GPU; returns the reference's 7-tuple."""
        if block_size != self.block_size or search_range != self.search_range:
            self.block_size, self.search_range = block_size, search_range
            self._engine = None
        eng = self.engine()
        cur = self._upload_padded(np.asarray(current_padded_frame))[0]
        refs = [self._upload_padded(np.asarray(r))[0] for r in ref_frames]
        qp_rd = self.Qp
        qp_row = self.row_qp_schedule(eng.nby) if self._rc_on() else None
        # frac frame wrap: the caller's list is uint8 unless it holds a float array
        wrap = all(np.asarray(r).dtype == np.uint8 for r in ref_frames)
        sym = eng.encode_p(cur, refs, qp_rd, qp_row, fme_wrap=wrap)
        if qp_row:
            self.set_Qp(qp_row[-1])
        return self._flow_tuple(sym, intra=False, stats=generate_row_wise_stats)

    def complete_intra_flow(self, current_padded_frame, intra_mode, block_size, search_range,
                            generate_row_wise_stats=True):
        """Encoder.py:1582-1642 on the GPU; returns the reference's 8-tuple."""
        if intra_mode != 0:
            raise NotImplementedError("only intra_mode 0 is built")
        if block_size != self.block_size or search_range != self.search_range:
            self.block_size, self.search_range = block_size, search_range
            self._engine = None
        eng = self.engine()
        cur = self._upload_padded(np.asarray(current_padded_frame))[0]
        qp_rd = self.Qp
        qp_row = self.row_qp_schedule(eng.nby) if self._rc_on() else None
        sym = eng.encode_i(cur, qp_rd, qp_row)
        if qp_row:
            self.set_Qp(qp_row[-1])
        return self._flow_tuple(sym, intra=True, stats=generate_row_wise_stats)

    def _flow_tuple(self, sym: FrameSymbols, intra: bool, stats: bool):
        host = symbols_to_host(sym)
        bs = self.block_size
        mvs = frame_mvs(host, bs)
        qblocks = frame_residuals(host, bs)
        avg_mae = self._avg_mae(host["mae_num"])
        recon = host["recon"][: self.h_pixels, : self.w_pixels]
        qp_row = sym.qp_row or []
        rsize = int(host["tokens"].sum())
        row_pct = []
        if stats:
            per_row = host["tokens"].reshape(-1, int(round(self.num_blocks_per_row))).sum(axis=1)
            row_pct = [(int(r) / rsize) * 100 for r in per_row] if rsize else []
        if intra:
            resid_frame = None
            return mvs, avg_mae, qblocks, qp_row, recon, resid_frame, rsize, row_pct
        return mvs, avg_mae, qblocks, qp_row, recon, rsize, row_pct

    def _avg_mae(self, mae_num: np.ndarray, bs: int | None = None) -> float:
        if (mae_num < 0).any():
            return float("inf")
        bs = self.block_size if bs is None else bs
        bb = bs * bs
        return (int(mae_num.astype(np.int64).sum()) / bb) / len(mae_num)

    # ---- GOP driver ------------------------------------------------------------------------
    def encode(self, intra_mode=None, intra_dur=None, search_range=None, block_size=None, save_enc_pkg=True):
        """Encoder.py:1790-1898.  Returns the PSNR per frame."""
        if search_range is not None and search_range != self.search_range:
            self.search_range, self._engine = search_range, None
        if block_size is not None and block_size != self.block_size:
            self.block_size, self._engine = block_size, None
            self.sub_block_size = block_size // 2
            self.num_blocks_per_row = self.w_pixels / block_size
        intra_dur = self.intra_dur if intra_dur is None else intra_dur
        intra_mode = self.intra_mode if intra_mode is None else intra_mode
        if intra_mode != 0:
            raise NotImplementedError("only intra_mode 0 is built")
        t0 = time.time()
        eng = self.engine()
        frames_dev = self._upload_padded(self.y_only_f_arr[: self.frames])
        result = self.encode_device(frames_dev, intra_dur)
        torch.cuda.synchronize(self.device)
        sse = result["sse"].cpu().numpy().astype(np.int64)
        hp, wp = eng.h, eng.w
        psnr_per_frame = [_psnr_from_sse(int(s), hp * wp) for s in sse]
        syms = result["symbols"]
        self._symbols = syms
        # closed-loop decode of the same symbols (Encoder.py:1873); result kept on device
        self.decoded_device = self.decoder.decode_symbols(syms, eng)
        pkg = LazyPackage(self, syms, psnr_per_frame, result["frame_type"], result["qp_rows"])
        if any("qp_map" in s.extra for s in syms):
            pkg["QP map per frame"] = [s.extra["qp_map"].cpu().numpy() if "qp_map" in s.extra else None for s in syms]
        self.encoded_package_f = True
        if save_enc_pkg:
            self.encoded_package = pkg
        self._save_recon(syms)
        self.inter0.append(time.time() - t0)
        return psnr_per_frame

    def encode_device(self, frames_dev: torch.Tensor, intra_dur: int, symbols=None, check: bool = True,
                      chunk: int | None = None, wait_input=None, on_output=None):
        """The GOP loop on device-resident frames [F, Hp, Wp].  Returns symbols per frame and
        a device SSE array.  check=True ends with one host read of the persistent runs'
        timeout count (Engine.check_run: raises if a dependency wait timed out); a caller
        that times back-to-back GOPs passes False and calls engine().check_run() after them.
        Otherwise no host sync unless RCFlag > 1 needs residual_size.

        Streaming hooks (hoststream.HostStreamEncoder): a persistent P-run covers at most
        `chunk` frames per launch; wait_input(k0, k1) is called before the work reading frames
        [k0, k1) is enqueued (to make the stream wait for their upload) and on_output(k0, k1,
        syms) after the work producing their symbols is enqueued.  Symbols are identical."""
        wait_input_default, on_output_default = wait_input is None, on_output is None
        wait_input = wait_input or (lambda k0, k1: None)
        on_output = on_output or (lambda k0, k1, syms: None)
        eng = self.engine()
        nframes = frames_dev.shape[0]
        # the reference's initial reference list: one all-128 frame (Encoder.py:1798), never
        # written, so one plane per engine serves every GOP (no fill per call)
        if getattr(eng, "_ref128", None) is None:
            eng._ref128 = alloc_planes(1, eng.h, eng.w, self.device, fill=128)[0]
        ref_frames = [eng._ref128]
        # the start frame is float64 in the reference (Encoder.py:1798): while it is in the
        # list the FME frac frame does not wrap its uint8 row sums (so_encode_p_rows_ex)
        ref_float = [True]
        out_syms, ftypes, qp_rows = [], [], []
        rc_on = self._rc_on()
        qp_sched = self.row_qp_schedule(eng.nby) if rc_on else None
        qp_sched_dev = eng.qp_row_tensor(qp_sched) if rc_on else None
        two_pass = self.RCFlag is not None and self.RCFlag >= 3
        roi = self.roi_block_offsets()
        roi_dev = eng.device_const_i32(roi) if roi is not None else None
        use_map = two_pass or roi_dev is not None
        lo, hi = self.qp_clamp

        def frame(cur, intra, qp_rd, out, wrap):
            """one frame: plain, ROI map, or two-pass (pass 1 -> so_qp_map -> pass 2)"""
            qmap = torch.empty(eng.nb, dtype=torch.int32, device=self.device) if use_map else None
            if intra:
                enc = lambda o, qm: eng.encode_i(cur, qp_rd, qp_sched, out=o, qp_row_dev=qp_sched_dev,  # noqa: E731
                                                 qp_map_dev=qm)
            else:
                enc = lambda o, qm, reuse=False, tok=False: eng.encode_p(  # noqa: E731
                    cur, ref_frames, qp_rd, qp_sched, out=o, qp_row_dev=qp_sched_dev, fme_wrap=wrap, qp_map_dev=qm,
                    **({"reuse_me": reuse} if reuse else {}), **({"tokens_only": tok} if tok else {}))
            if two_pass:
                # pass 1 needs only the token counts (and the ME records pass 2 reuses)
                sym = enc(out, None) if intra else enc(out, None, tok=True)
                eng.qp_map(sym.tokens, qp_rd, qp_sched_dev, roi_dev, qmap, qp_lo=lo, qp_hi=hi)
                sym = enc(sym, qmap) if intra else enc(sym, qmap, True)
            elif roi_dev is not None:
                eng.qp_map(None, qp_rd, qp_sched_dev, roi_dev, qmap, qp_lo=lo, qp_hi=hi)
                sym = enc(out, qmap)
            else:
                sym = enc(out, None)
            if qmap is not None:
                sym.extra["qp_map"] = qmap
            return sym

        rc_switch = self.RCFlag is not None and self.RCFlag > 1 and (self.RCFlag == 2 or self.intra_thresh is not None)
        # runs of P-frames with nothing per frame on the host go through one persistent launch
        # (engine.encode_p_run): same symbols, frames overlapped on the device
        run_ok = not rc_switch and self.nRefFrames == 1 and eng.pipelined_ok(1) and os.environ.get("SO_PIPELINE", "1") != "0"
        pipelined = run_ok and not two_pass and roi_dev is None
        # two-pass RC (with or without ROI): a P-run in one so_encode_p_run_2pass call -- both
        # passes of every frame in one persistent launch (default; SO_OPT_RUN_2PASS_FUSED = 0: the
        # per-frame kernel sequence enqueued by the library), pass 1 with the previous frame's
        # motion records as its search hint, which the per-call C-ABI of the loop below has no
        # argument for (SO_RUN_2PASS=0: the loop)
        pipelined2 = (run_ok and two_pass and eng.pipelined_ok(1, vbs_ok=False)
                      and os.environ.get("SO_RUN_2PASS", "1") == "1")
        if pipelined and chunk is None and intra_dur < nframes - 1 and wait_input_default and on_output_default:
            # several P-runs between I-frames: independent chains, interleaved in one launch
            return self.encode_gops_device([frames_dev], intra_dur, symbols=[symbols] if symbols else None,
                                           check=check)[0]
        i = 0
        while i < nframes:
            if (pipelined or pipelined2) and i % intra_dur != 0:
                j = i
                while j < nframes and j % intra_dur != 0 and (chunk is None or j - i < chunk):
                    j += 1
                wait_input(i, j)
                self.set_Qp(self.const_init_Qp)
                outs = []
                for k in range(i, j):
                    pre = symbols[k] if symbols is not None else None
                    outs.append(pre if pre is not None and pre.frame_type == 1 else eng.new_symbols(1))
                if pipelined2:
                    maps = [o.extra["qp_map"] if "qp_map" in o.extra else
                            torch.empty(eng.nb, dtype=torch.int32, device=self.device) for o in outs]
                    eng.encode_p_run_2pass([frames_dev[k] for k in range(i, j)], ref_frames[-1], self.Qp, outs, maps,
                                           qp_row=qp_sched, qp_row_dev=qp_sched_dev, roi_dev=roi_dev, qp_lo=lo,
                                           qp_hi=hi)
                else:
                    eng.encode_p_run([frames_dev[k] for k in range(i, j)], ref_frames[-1], self.Qp, outs,
                                     qp_row=qp_sched, qp_row_dev=qp_sched_dev)
                for sym in outs:
                    out_syms.append(sym)
                    ftypes.append(1)
                    qp_rows.append(list(qp_sched) if rc_on else [])
                if rc_on:
                    self.set_Qp(qp_sched[-1])
                ref_frames = [outs[-1].recon]
                ref_float = [False]
                on_output(i, j, outs)
                i = j
                continue
            wait_input(i, i + 1)
            cur = frames_dev[i]
            pre = symbols[i] if symbols is not None else None
            self.set_Qp(self.const_init_Qp)
            if i % intra_dur == 0:
                sym = frame(cur, True, self.Qp, pre if pre is not None and pre.frame_type == 0 else None, True)
            else:
                sym = frame(cur, False, self.Qp, pre if pre is not None and pre.frame_type == 1 else None,
                            not any(ref_float))
                # RCFlag 2 (and 3 given an intra_thresh): P->I switch on the residual size,
                # one host read per P-frame (Encoder.py:1851-1856)
                if self.RCFlag is not None and self.RCFlag > 1 and (self.RCFlag == 2 or self.intra_thresh is not None):
                    residual_size = int(sym.tokens.sum().item())
                    if residual_size > self.intra_thresh:
                        # self.Q still holds the last row's QP of the inter pass (quirk
                        # of Encoder.py:1851-1856 after the per-row set_Qp calls)
                        sym = frame(cur, True, qp_sched[-1], None, True)
            if rc_on:
                self.set_Qp(qp_sched[-1])
            out_syms.append(sym)
            ftypes.append(sym.frame_type)
            qp_rows.append(list(qp_sched) if rc_on else [])
            on_output(i, i + 1, [sym])
            if i < nframes - 1:
                if len(ref_frames) >= self.nRefFrames:
                    ref_frames.pop(0)
                    ref_float.pop(0)
                ref_frames.append(sym.recon)
                ref_float.append(False)
            i += 1
        # per-block / per-row SSE came out of the encode kernels; one reduction per GOP
        sse = eng.sum_rows([s.sse for s in out_syms])
        if check and (pipelined or pipelined2):
            eng.check_run()
        return {"symbols": out_syms, "sse": sse, "frame_type": ftypes, "qp_rows": qp_rows}

    def encode_gops_device(self, gops: list, intra_dur: int, symbols=None, check: bool = True) -> list:
        """Several GOPs (device-resident [F, Hp, Wp] each, e.g. consecutive GOPs of one stream
        or GOPs of different streams) encoded together: every I-frame first (they depend on
        nothing), then the P-frame runs of ALL the GOPs interleaved in one persistent launch
        (Engine.encode_p_runs), so a frame of each run is in flight at once.  Where one frame
        has fewer tiles than the GPU has resident workgroups (1080p) one GOP's frame-to-frame
        dependency leaves CUs idle that the other GOPs fill.  Each GOP's symbols are identical
        to encode_device of that GOP alone (the reference's encode() loop, Encoder.py:1839-1867,
        once per GOP).  Covers the persistent-run configuration (no two-pass RC / ROI / RCFlag>1
        P->I switch, nRefFrames 1); returns one encode_device-style dict per GOP.
        symbols: optional per-GOP lists of preallocated FrameSymbols to reuse."""
        eng = self.engine()
        rc_switch = self.RCFlag is not None and self.RCFlag > 1 and (self.RCFlag == 2 or self.intra_thresh is not None)
        if not (eng.pipelined_ok(1) and self.nRefFrames == 1 and not rc_switch and self.roi_block_offsets() is None
                and not (self.RCFlag is not None and self.RCFlag >= 3)):
            raise ValueError("encode_gops_device covers the persistent-run configuration only")
        rc_on = self._rc_on()
        qp_sched = self.row_qp_schedule(eng.nby) if rc_on else None
        qp_sched_dev = eng.qp_row_tensor(qp_sched) if rc_on else None
        self.set_Qp(self.const_init_Qp)
        qp = self.Qp
        outs, runs = [], []
        for g, frames_dev in enumerate(gops):
            n = frames_dev.shape[0]
            pre = symbols[g] if symbols is not None else [None] * n
            syms = [None] * n
            for i in range(0, n, intra_dur):   # the I-frames
                p = pre[i] if pre[i] is not None and pre[i].frame_type == 0 else None
                syms[i] = eng.encode_i(frames_dev[i], qp, qp_sched, out=p, qp_row_dev=qp_sched_dev)
            for i in range(0, n, intra_dur):   # the P-runs after each of them
                ks = list(range(i + 1, min(i + intra_dur, n)))
                for k in ks:
                    syms[k] = pre[k] if pre[k] is not None and pre[k].frame_type == 1 else eng.new_symbols(1)
                if ks:
                    runs.append(([frames_dev[k] for k in ks], syms[i].recon, [syms[k] for k in ks]))
            outs.append(syms)
        eng.encode_p_runs(runs, qp, qp_row=qp_sched, qp_row_dev=qp_sched_dev)
        if rc_on:   # the state encode_device leaves (each frame ends on its last row's QP)
            self.set_Qp(qp_sched[-1])
        res = []
        for syms in outs:
            res.append({"symbols": syms, "sse": eng.sum_rows([s.sse for s in syms]),
                        "frame_type": [s.frame_type for s in syms],
                        "qp_rows": [list(qp_sched) if rc_on else [] for _ in syms]})
        if check:
            eng.check_run()
        return res

    def _save_recon(self, syms):
        d = os.path.dirname(self.recon_yuv_path)
        if d and not os.path.isdir(d):
            return  # the reference would raise here; writing the file is host I/O, not the path
        with open(self.recon_yuv_path, "wb") as f:
            for s in syms:
                f.write(s.recon.cpu().numpy()[: self.h_pixels, : self.w_pixels].tobytes())

    def save_y_only(self, filename, y_data_list):
        with open(filename, "wb") as f:
            for data in y_data_list:
                f.write(np.asarray(data).tobytes())

    def get_encoded_package(self):
        return self.encoded_package

    def transmit_packed(self, path: str) -> int:
        """The encoded GOP as one binary file of packed symbols (packedfile.py: varint split /
        MVs / RLE token lists packed on the GPU by so_pack_frames, ~2.4x smaller than the
        int16 QTC and far smaller than the text lines).  decoder.decode_packed_file reads it.
        Returns the file size in bytes."""
        if not self.encoded_package_f or self._symbols is None:
            print("[ERROR] No encoded package available, please run encode() first")
            return 0
        from . import packedfile
        return packedfile.write(path, self.engine(), self._symbols, self.encoded_package["Qp_per_row_per_frame"])

    def transmit_bitstream(self, intra_dur=None, block_size=None, mv_file=None, residual_file=None,
                           qp_map_file=None):
        """Encoder.py:1544-1573, writing the differential MV/QP lines and the RLE residual
        lines (entropy_encoder_frame) — the reference writes str(residuals) instead, which
        its own parser cannot read.  With ROI / two-pass RC (build extension)
        `qp_map_file` receives one line per frame of per-block QP deltas against the row QP."""
        if not self.encoded_package_f:
            print("[ERROR] No encoded package available, please run encode() first")
            return
        pkg = self.encoded_package
        with open(mv_file, "w") as fm, open(residual_file, "w") as fr:
            for i in range(len(pkg["MVS per Frame"])):
                ft = pkg["frame_type_seq"][i]
                fm.write(str(ft) + "|" + self.differential_encoder_frame(ft, pkg["MVS per Frame"][i],
                                                                         pkg["Qp_per_row_per_frame"][i]) + "\n")
                fr.write(self.entropy_encoder_frame(pkg["approx residual"][i], block_size or self.block_size) + "\n")
        if qp_map_file is not None:
            from .bitstream import qp_map_line
            maps = pkg["QP map per frame"] if "QP map per frame" in pkg else None
            with open(qp_map_file, "w") as fq:
                for i in range(len(pkg["frame_type_seq"])):
                    m = maps[i] if maps is not None else None
                    fq.write(("" if m is None else qp_map_line(m, pkg["Qp_per_row_per_frame"][i], self.const_init_Qp,
                                                                self.num_blocks_per_row)) + "\n")
