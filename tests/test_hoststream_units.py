"""Host logic of hoststream.HostStreamEncoder (no GPU): the encode units its uploads follow
must be the frame ranges Y_Video_codec.encode_device works on in turn (each I-frame alone, the
P-runs of at most `chunk` frames between I-frames), and the packed views slice the page-locked
buffer at the downloaded lengths."""
from types import SimpleNamespace

import pytest
import torch

from streamoptima_amd.hoststream import HostStreamEncoder, _PackedViews


def _encode_device_units(nframes, intra_dur, chunk):
    """The unit sequence of encode_device's loop (Encoder.py's GOP driver, pipelined P-runs)."""
    out, i = [], 0
    while i < nframes:
        if i % intra_dur != 0:
            j = i
            while j < nframes and j % intra_dur != 0 and j - i < chunk:
                j += 1
            out.append((i, j))
            i = j
        else:
            out.append((i, i + 1))
            i += 1
    return out


@pytest.mark.parametrize("nframes,intra_dur,chunk", [(30, 30, 2), (30, 30, 3), (8, 4, 3), (7, 7, 2), (5, 1, 2),
                                                     (12, 5, 4), (1, 1, 2), (30, 30, 29)])
def test_units_follow_encode_device(nframes, intra_dur, chunk):
    units = HostStreamEncoder._units(SimpleNamespace(nframes=nframes, chunk=chunk), intra_dur)
    assert units == _encode_device_units(nframes, intra_dur, chunk)
    assert [f for a, b in units for f in range(a, b)] == list(range(nframes))   # every frame once, in order


def test_packed_views_slice_at_lengths():
    buf = torch.arange(4 * 10, dtype=torch.int64).view(4, 10).to(torch.uint8)
    v = _PackedViews(buf, [3, 0, 10, 7])
    assert len(v) == 4
    assert v[0].tolist() == [0, 1, 2] and v[1].numel() == 0 and v[2].numel() == 10
    assert [t.numel() for t in v] == [3, 0, 10, 7]
    assert v[3].data_ptr() == buf[3].data_ptr()   # a view, not a copy
