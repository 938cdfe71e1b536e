"""Drop-in `decoder` (the reference's decoder.py surface) on the MI355X path.

decode() reconstructs frames from symbols with the same gfx950 kernels as the encoder's
reconstruction (decoder.py:97-211 inter, :330-432 intra mode 0, :487-545 GOP loop incl.
its reference-list handling: an I-frame CLEARS the list, decoder.py:520).  With
FMEEnable the references are the frac frames (decoder.py:102-103, 468-483); after the
I-frame reset the list holds uint8 reconstructions only, so their row sums always wrap.
"""
from __future__ import annotations

import numpy as np
import torch

from . import bitstream as _bs
from .bitstream import entropy_encoder_block  # noqa: F401  (API parity helpers live there)
from .engine import Engine, alloc_planes


def _canon_frame(frame_type, mvs, residuals, bs):
    """reference per-block lists -> canonical arrays (split, mv, qtc)."""
    nb = len(mvs)
    split = np.zeros(nb, np.uint8)
    qtc = np.zeros((nb, bs * bs), np.int16)
    mv = np.zeros((nb, 4, 3) if frame_type == 1 else (nb, 4), np.int16)
    sb2 = (bs // 2) ** 2
    for i, (m, r) in enumerate(zip(mvs, residuals)):
        if m[0] == 0:
            mv[i, 0] = m[1]
            qtc[i] = np.asarray(r[1]).reshape(-1)
        else:
            split[i] = 1
            for j in range(4):
                mv[i, j] = m[1][j]
                qtc[i, j * sb2:(j + 1) * sb2] = np.asarray(r[1][j]).reshape(-1)
    return split, mv, qtc


class decoder:
    def __init__(self, intra_mode, intra_dur, block_size, frames, height, width, Qp, nRefFrames, FMEEnable, lam,
                 VBSEnable, VBSoverlay=None, RCFlag=None, targetBR=None, frame_rate=30, qp_rate_tables=None,
                 ParallelMode=0, device=None):
        self.intra_mode = intra_mode
        self.intra_dur = intra_dur
        self.block_size = block_size
        self.sub_block_size = block_size // 2
        self.frames = frames
        self.h_pixels = height
        self.w_pixels = width
        self.num_blocks_per_row = width / block_size
        self.decoded_vid = None
        self.decoded_vid_f = False
        self.Qp = Qp
        self.nRefFrames = nRefFrames
        self.FMEEnable = FMEEnable
        self.lam = lam
        self.VBSEnable = VBSEnable
        self.VBSoverlay = VBSoverlay
        self.RCFlag = RCFlag
        self.frame_rate = frame_rate
        self.qr_rate_tables = qp_rate_tables
        self.ParallelMode = ParallelMode
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self._engine = None

    def _eng(self, engine=None) -> Engine:
        if engine is not None:
            return engine
        bs = self.block_size
        hp = -(-self.h_pixels // bs) * bs
        wp = -(-self.w_pixels // bs) * bs
        if self._engine is None:
            self._engine = Engine(hp, wp, bs, 16, False, 0.0, self.device, fme=bool(self.FMEEnable))
        return self._engine

    def _rc(self):
        return self.RCFlag is not None and self.RCFlag > 0

    def decode_symbols(self, symbols, engine=None):
        """GOP decode straight from device symbols (the encoder's closed loop)."""
        eng = self._eng(engine)
        ref_frames = [alloc_planes(1, eng.h, eng.w, eng.device, fill=128)[0]]
        out = []
        n = len(symbols)
        for i, s in enumerate(symbols):
            qp_row = s.qp_row if self._rc() else None
            qm = s.extra.get("qp_map")      # ROI / two-pass per-block QP (build extension)
            if s.frame_type == 0:
                rec = eng.recon_intra(s.split, s.mv, s.qtc, self.Qp, qp_row, qp_map_dev=qm)
                ref_frames = []
            else:
                rec = eng.recon_inter(ref_frames, s.split, s.mv, s.qtc, self.Qp, qp_row, qp_map_dev=qm)
            out.append(rec)
            if i < n - 1:
                if len(ref_frames) >= self.nRefFrames:
                    ref_frames.pop(0)
                ref_frames.append(rec)
        return out

    def decode(self, frame_type_seq, residual_file, Qp_per_row_per_frame, mv_file, intra_mode=None, intra_dur=None,
               block_size=None, frames=None, width=None, height=None, save_decoded_frames=True, qp_maps=None):
        """decoder.py:487-545 with the per-frame lists of the encoded package.  qp_maps: per
        frame per-block QPs (ROI / two-pass RC build extension) or None."""
        bs = block_size or self.block_size
        frames = frames or self.frames
        eng = self._eng()
        ref_frames = [alloc_planes(1, eng.h, eng.w, eng.device, fill=128)[0]]
        decoded = []
        for i in range(frames):
            ft = frame_type_seq[i]
            split, mv, qtc = _canon_frame(ft, mv_file[i], residual_file[i], bs)
            split_d = torch.from_numpy(split).to(eng.device)
            mv_d = torch.from_numpy(mv).to(eng.device)
            qtc_d = torch.from_numpy(qtc).to(eng.device)
            qp_row = Qp_per_row_per_frame[i] if self._rc() else None
            qm = None
            if qp_maps is not None and qp_maps[i] is not None:
                qm = torch.as_tensor(np.asarray(qp_maps[i], np.int32)).to(eng.device)
            if ft == 0:
                rec = eng.recon_intra(split_d, mv_d, qtc_d, self.Qp, qp_row, qp_map_dev=qm)
                ref_frames = []
            else:
                rec = eng.recon_inter(ref_frames, split_d, mv_d, qtc_d, self.Qp, qp_row, qp_map_dev=qm)
            decoded.append(rec)
            if i < frames - 1:
                if len(ref_frames) >= self.nRefFrames:
                    ref_frames.pop(0)
                ref_frames.append(rec)
        host = [d.cpu().numpy()[: self.h_pixels, : self.w_pixels] for d in decoded]
        if save_decoded_frames:
            self.decoded_vid_f = True
            self.decoded_vid = host
        return host

    # ---- text bitstream (decoder.py:547-710) ----------------------------------------------
    def entropy_decoder_block(self, encoded_block, block_size):
        return _bs.entropy_decoder_block(encoded_block, block_size)

    def differential_decoder_frame(self, mv_for_frame):
        return _bs.differential_decoder_frame(mv_for_frame, self.RCFlag, self.num_blocks_per_row)

    def entropy_decoder_frame(self, residual_for_frame, block_size):
        return _bs.entropy_decoder_frame(residual_for_frame, block_size)

    def decode_differential_entropy(self, all_mv_f, all_residual_f, block_size):
        """decoder.py:666-684: the two text files -> per-frame symbol lists."""
        frame_type_seq, mv_for_vid, qp_for_vid, res_for_vid = [], [], [], []
        with open(all_mv_f) as f:
            for line in f:
                ft, mvs, qps = self.differential_decoder_frame(line)
                frame_type_seq.append(ft)
                mv_for_vid.append(mvs)
                qp_for_vid.append(qps)
        with open(all_residual_f) as f:
            for line in f:
                res_for_vid.append(self.entropy_decoder_frame(line, block_size))
        return frame_type_seq, mv_for_vid, qp_for_vid, res_for_vid

    def decode_bitstream(self, mv_file, residual_file, intra_mode=None, intra_dur=None, block_size=None, frames=None,
                         width=None, height=None, save_decoded_frames=True, qp_map_file=None):
        """decoder.py:686-709: parse the transmitted text bitstream (transmit_bitstream)
        on the host, reconstruct every frame on the GPU.  qp_map_file: the per-block QP
        lines of ROI / two-pass RC (build extension)."""
        bs = block_size or self.block_size
        ft, mvs, qps, res = self.decode_differential_entropy(mv_file, residual_file, bs)
        self.mv_per_frame = mvs
        self.residuals_per_frame = res
        maps = None
        if qp_map_file is not None:
            with open(qp_map_file) as f:
                maps = [(_bs.parse_qp_map_line(line, qps[i] if self._rc() else None, self.Qp, self.num_blocks_per_row)
                         if line.strip() else None) for i, line in enumerate(f)]
        return self.decode(ft, res, qps, mvs, intra_mode, intra_dur, bs, frames, width, height, save_decoded_frames,
                           qp_maps=maps)

    def decode_packed_file(self, path: str, save_decoded_frames=True):
        """Encoder.transmit_packed's file: the packed streams go to the GPU, so_unpack_frames
        restores split / mv / qtc of every block in parallel, and the frames are rebuilt by the
        same kernels as decode()."""
        from . import packedfile
        eng = self._eng()
        meta = packedfile.read(path, eng.device)
        if (meta["h"], meta["w"], meta["bs"], meta["nb"]) != (eng.h, eng.w, eng.bs, eng.nb):
            raise ValueError(f"{path}: {meta['w']}x{meta['h']} bs {meta['bs']} does not match this decoder")
        syms = eng.unpack_symbols(meta["frame_types"], meta["packed"], meta["offs"])
        for s, q in zip(syms, meta["qp_rows"]):
            s.qp_row = q or None
        decoded = self.decode_symbols(syms, eng)
        host = [d.cpu().numpy()[: self.h_pixels, : self.w_pixels] for d in decoded]
        if save_decoded_frames:
            self.decoded_vid_f = True
            self.decoded_vid = host
        return host

    def save_decoded_frames(self, filename="yuv/decoded_bitstream_frames.yuv"):
        if not self.decoded_vid_f:
            print("[ERROR] No decoded frames available.")
            return
        with open(filename, "wb") as f:
            for data in self.decoded_vid:
                f.write(data.tobytes())
