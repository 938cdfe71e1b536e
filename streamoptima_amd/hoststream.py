"""Host-to-host GOP encode with the transfers overlapped (BASELINE.md §4's timed region:
pinned host Y planes in, symbols out).

The reference reads frames from host memory and writes its bitstream text to files
(Encoder.py:1790-1898, transmit_bitstream :1544-1580).  Here the three engines of the card
work at once:

    copy stream A (H2D)   frame 0 | frames 1..C | frames C+1..2C | ...
    compute stream        I-frame | P-run 1..C (+ pack) | P-run C+1..2C (+ pack) | ...
    copy stream B (D2H)                  packed chunk 0 | packed chunk 1 | ...

A P-run chunk waits for its frames' upload events only; the packed symbol stream of a chunk
(Engine.pack_symbols: varint split / MVs / RLE token lists, 2.4x smaller than the int16
QTC) is downloaded as soon as its byte counts are known, while the next chunk encodes.
The host waits for a chunk's byte counts only after it has enqueued the following chunk, so
the compute stream never idles on the host.  Symbols are those of encode_device (the chunks
are persistent P-runs with the previous chunk's reconstruction as their reference).
"""
from __future__ import annotations

import torch

from .engine import alloc_planes


class HostStreamEncoder:
    def __init__(self, codec, nframes: int, chunk: int = 2):
        eng = codec.engine()
        self.codec, self.eng, self.nframes, self.chunk = codec, eng, int(nframes), int(chunk)
        dev = codec.device
        self.dev = dev
        self.frames_dev = alloc_planes(self.nframes, eng.h, eng.w, dev)
        self.h2d = torch.cuda.Stream(dev)
        self.d2h = torch.cuda.Stream(dev)
        self.syms = None
        self.offs = torch.empty((self.nframes, eng.nb + 1), dtype=torch.int32, device=dev)
        self.packed = torch.empty((self.nframes, eng.pack_bound()), dtype=torch.uint8, device=dev)
        self.tot_h = torch.empty(self.nframes, dtype=torch.int32).pin_memory()
        self.packed_h = torch.empty(self.packed.shape, dtype=torch.uint8).pin_memory()
        self.sse_h = torch.empty(self.nframes, dtype=torch.int64).pin_memory()

    def encode(self, frames_host: torch.Tensor, intra_dur: int) -> dict:
        """frames_host: pinned uint8 [F, Hp, Wp].  Returns {"packed": [host uint8 view per
        frame], "bytes": [...], "sse": host int64 [F], "frame_type": [...]} once everything
        is in host memory."""
        f = self.nframes
        if tuple(frames_host.shape) != tuple(self.frames_dev.shape) or not frames_host.is_pinned():
            raise ValueError("frames_host must be pinned uint8 of the encoder's padded frame shape")
        eng, comp = self.eng, torch.cuda.current_stream(self.dev)
        if self.syms is None:
            self.syms = [eng.new_symbols(0 if i % intra_dur == 0 else 1) for i in range(f)]
        up = []
        with torch.cuda.stream(self.h2d):
            self.h2d.wait_stream(comp)        # the previous GOP's reads of frames_dev are done
            for i in range(f):
                self.frames_dev[i].copy_(frames_host[i], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.h2d)
                up.append(ev)
        pending = []

        def drain(upto_len):
            while len(pending) > upto_len:
                k0, k1, ev = pending.pop(0)
                ev.synchronize()                    # byte counts of frames [k0, k1) are in tot_h
                self.d2h.wait_event(ev)
                with torch.cuda.stream(self.d2h):
                    for i in range(k0, k1):
                        n = int(self.tot_h[i])
                        self.packed_h[i, :n].copy_(self.packed[i, :n], non_blocking=True)

        def wait_input(k0, k1):
            comp.wait_event(up[k1 - 1])

        def on_output(k0, k1, syms):
            eng.pack_symbols(syms, self.offs[k0:k1], self.packed[k0:k1])
            self.tot_h[k0:k1].copy_(self.offs[k0:k1, eng.nb], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(comp)
            pending.append((k0, k1, ev))
            drain(1)                                 # the chunk before this one

        res = self.codec.encode_device(self.frames_dev, intra_dur, symbols=self.syms, check=False, chunk=self.chunk,
                                       wait_input=wait_input, on_output=on_output)
        self.sse_h.copy_(res["sse"], non_blocking=True)
        drain(0)
        comp.synchronize()
        self.d2h.synchronize()
        eng.check_run()
        nbytes = self.tot_h.tolist()
        return {"packed": [self.packed_h[i, :n] for i, n in enumerate(nbytes)], "bytes": nbytes,
                "sse": self.sse_h.clone(), "frame_type": res["frame_type"]}
