"""Host-to-host GOP encode with the transfers overlapped (BASELINE.md §4's timed region:
pinned host Y planes in, symbols out).

The reference reads frames from host memory and writes its bitstream text to files
(Encoder.py:1790-1898, transmit_bitstream :1544-1580).  Here the three engines of the card
work at once:

    copy stream A (H2D)   frame 0 | frames 1..C | frames C+1..2C | ... | next GOP's frames ...
    compute stream        I-frame | P-run 1..C (+ pack) | P-run C+1..2C (+ pack) | ...
    copy stream B (D2H)                  packed chunk 0 | packed chunk 1 | ...

A P-run chunk waits for its frames' upload events only; the packed symbol stream of a chunk
(Engine.pack_symbols: varint split / MVs / RLE token lists, 2.4x smaller than the int16
QTC) is downloaded as soon as its byte counts are known, while the next chunk encodes.
The host waits for a chunk's byte counts only after it has enqueued the following chunk, so
the compute stream never idles on the host.  Symbols are those of encode_device (the chunks
are persistent P-runs with the previous chunk's reconstruction as their reference).

encode_stream() runs several GOPs back to back with two sets of frame / packed buffers: the
next GOP's upload is queued before the current GOP encodes, so the H2D engine never waits for
the compute stream (a GOP then costs about its upload time).
"""
from __future__ import annotations

import time

import torch

from .engine import alloc_planes
from .hostmem import device_ptr, pinned_empty
from .hwqueue import dedicated_stream


class _Buffers:
    """One GOP in flight: device frames, packed streams and their pinned host copies."""

    def __init__(self, eng, nframes: int, dev):
        self.frames_dev = alloc_planes(nframes, eng.h, eng.w, dev)
        self.offs = torch.empty((nframes, eng.nb + 1), dtype=torch.int32, device=dev)
        self.packed = torch.empty((nframes, eng.pack_bound()), dtype=torch.uint8, device=dev)
        self.tot_h = pinned_empty((nframes,), torch.int32)
        self.tot_dptr = device_ptr(self.tot_h)     # the pack's scan stores each frame's length here
        self.packed_h = pinned_empty(tuple(self.packed.shape))
        self.sse_h = pinned_empty((nframes,), torch.int64)
        self.enc_done = None      # compute-stream event: this set's frames are no longer read
        self.d2h_done = None      # D2H-stream event: this set's packed streams are downloaded
        self.gop = None           # (index, frame types) of the GOP it holds


class _PackedViews:
    """Frame i's packed stream as packed_h[i, :bytes[i]], made when asked for."""

    def __init__(self, packed_h, nbytes):
        self._p, self._n = packed_h, nbytes

    def __len__(self):
        return len(self._n)

    def __getitem__(self, i):
        return self._p[i, :self._n[i]]

    def __iter__(self):
        return (self[i] for i in range(len(self._n)))


class HostStreamEncoder:
    def __init__(self, codec, nframes: int, chunk: int = 2, nbuf: int = 1, upload: str = "chunk"):
        """upload: "chunk" = one H2D copy per encode unit (the I-frame, each P-run chunk), "frame"
        = one per frame."""
        eng = codec.engine()
        self.codec, self.eng, self.nframes, self.chunk = codec, eng, int(nframes), int(chunk)
        if upload not in ("chunk", "frame"):
            raise ValueError("upload must be 'chunk' or 'frame'")
        self.upload = upload
        self.dev = codec.device
        # the three engines' streams each on a hardware queue of its own (hwqueue.py): on a
        # shared queue a stream's event wait stalls the others and the region runs serially
        self.h2d = dedicated_stream(self.dev, "hoststream.h2d")
        self.d2h = dedicated_stream(self.dev, "hoststream.d2h")
        self.comp = dedicated_stream(self.dev, "hoststream.compute")
        self.syms = None
        self.bufs = [_Buffers(eng, self.nframes, self.dev) for _ in range(max(1, int(nbuf)))]

    @property
    def frames_dev(self):
        return self.bufs[0].frames_dev

    def _check(self, frames_host):
        if tuple(frames_host.shape) != tuple(self.bufs[0].frames_dev.shape) or not frames_host.is_pinned():
            raise ValueError("frames_host must be pinned uint8 of the encoder's padded frame shape")

    def _units(self, intra_dur: int) -> list:
        """The frame ranges encode_device works on in turn: each I-frame, and the P-runs of at
        most `chunk` frames between them."""
        r, i = [], 0
        while i < self.nframes:
            j = i + 1
            if i % intra_dur != 0:
                while j < self.nframes and j % intra_dur != 0 and j - i < self.chunk:
                    j += 1
            r.append((i, j))
            i = j
        return r

    def _upload(self, b: _Buffers, frames_host, intra_dur: int) -> list:
        """Queue the GOP's upload; returns per frame the event after the copy that carries it
        (one copy per encode unit: 16.6 MB copies ran at 52.6 GB/s, 8.3 MB ones at 50.0 on the
        GPU box, tools/s4_links.py)."""
        up = [None] * self.nframes
        units = self._units(intra_dur) if self.upload == "chunk" else [(i, i + 1) for i in range(self.nframes)]
        with torch.cuda.stream(self.h2d):
            if b.enc_done is not None:
                self.h2d.wait_event(b.enc_done)      # the GOP that last used these frames is encoded
            for k0, k1 in units:
                b.frames_dev[k0:k1].copy_(frames_host[k0:k1], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.h2d)
                up[k0:k1] = [ev] * (k1 - k0)
        return up

    def _result(self, b: _Buffers) -> dict:
        nbytes = b.tot_h.tolist()
        return {"packed": _PackedViews(b.packed_h, nbytes), "bytes": nbytes,
                "sse": b.sse_h.clone(), "frame_type": b.gop[1]}

    def encode(self, frames_host: torch.Tensor, intra_dur: int) -> dict:
        """frames_host: pinned uint8 [F, Hp, Wp].  Returns {"packed": [host uint8 view per
        frame], "bytes": [...], "sse": host int64 [F], "frame_type": [...]} once everything
        is in host memory (the views stay valid until the next call)."""
        out = []
        self.encode_stream([frames_host], intra_dur, lambda k, r: out.append(r))
        return out[0]

    def encode_stream(self, gops: list, intra_dur: int, consume, trace: list | None = None) -> None:
        """Encode GOPs back to back; consume(k, result) is called for GOP k, in order, once its
        symbols are in host memory and before its buffers are reused (the result's views are
        valid only inside the call).  With two buffer sets (nbuf=2) GOP k+1's upload runs
        during GOP k's encode."""
        for g in gops:
            self._check(g)
        caller = torch.cuda.current_stream(self.dev)
        self.comp.wait_stream(caller)       # the caller's earlier work on the inputs / buffers
        with torch.cuda.stream(self.comp):
            self._encode_stream(gops, intra_dur, consume, trace)

    def _encode_stream(self, gops: list, intra_dur: int, consume, trace) -> None:
        eng, comp, nb = self.eng, self.comp, len(self.bufs)
        if self.syms is None:
            self.syms = [eng.new_symbols(0 if i % intra_dur == 0 else 1) for i in range(self.nframes)]
        pending, waiting = [], []      # chunks whose byte counts are on their way; finished GOPs

        def mark(label, stream):       # tools/stream_probe.py: (label, event, host time)
            if trace is not None:
                ev = torch.cuda.Event(enable_timing=True)
                ev.record(stream)
                trace.append((label, ev, time.perf_counter()))

        def drain(upto_len):
            while len(pending) > upto_len:
                b, k0, k1, ev = pending.pop(0)
                ev.synchronize()                    # byte counts of frames [k0, k1) are in tot_h
                self.d2h.wait_event(ev)
                mark(f"d2h_go {k0}", self.d2h)
                with torch.cuda.stream(self.d2h):
                    for i in range(k0, k1):
                        n = int(b.tot_h[i])
                        b.packed_h[i, :n].copy_(b.packed[i, :n], non_blocking=True)
                if k1 == self.nframes:              # the GOP's last chunk: its download is queued
                    b.d2h_done = torch.cuda.Event()
                    b.d2h_done.record(self.d2h)
                    mark(f"d2h_end {b.gop[0] if b.gop else '?'}", self.d2h)

        def retire(b):
            """Hand GOP b.gop to the caller (its chunks all drained) and free the set."""
            if any(p[0] is b for p in pending):
                drain(0)
            while waiting and waiting[0] is b:
                waiting.pop(0)
                b.enc_done.synchronize()            # its SSE copy (compute stream)
                b.d2h_done.synchronize()            # its packed streams (D2H stream)
                consume(b.gop[0], self._result(b))
                b.gop = None

        ups = {}
        for k, g in enumerate(gops):
            b = self.bufs[k % nb]
            if b.gop is not None:
                retire(b)                            # GOP k - nb: long finished when nb > 1
            if k == 0 or nb == 1:
                ups[k] = self._upload(b, g, intra_dur)
                mark(f"up_end {k}", self.h2d)
            if nb > 1 and k + 1 < len(gops):       # the next GOP's upload, queued before this encode
                ups[k + 1] = self._upload(self.bufs[(k + 1) % nb], gops[k + 1], intra_dur)
                mark(f"up_end {k + 1}", self.h2d)
            up = ups.pop(k)
            if b.d2h_done is not None:
                comp.wait_event(b.d2h_done)         # this set's previous packed streams are down
            b.gop = (k, None)
            mark(f"enc_start {k}", comp)

            def wait_input(k0, k1, up=up):
                comp.wait_event(up[k1 - 1])
                mark(f"chunk_go {k0}", comp)

            def on_output(k0, k1, syms, b=b):
                # the scan stores the frames' lengths straight into tot_h (so_pack_frames_ex)
                eng.pack_symbols(syms, b.offs[k0:k1], b.packed[k0:k1], totals_ptr=b.tot_dptr + 4 * k0)
                ev = torch.cuda.Event()
                ev.record(comp)
                mark(f"chunk_end {k0}", comp)
                pending.append((b, k0, k1, ev))
                drain(1)                             # the chunk before this one

            res = self.codec.encode_device(b.frames_dev, intra_dur, symbols=self.syms, check=False,
                                           chunk=self.chunk, wait_input=wait_input, on_output=on_output)
            b.sse_h.copy_(res["sse"], non_blocking=True)
            b.enc_done = torch.cuda.Event()
            b.enc_done.record(comp)
            mark(f"enc_end {k}", comp)
            b.gop = (k, res["frame_type"])
            waiting.append(b)
        drain(0)
        for b in list(waiting):
            retire(b)
        comp.synchronize()
        eng.check_run(defer_stats=True)
