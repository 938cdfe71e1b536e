"""The benchmarked workloads (BASELINE.json `configs`), in one place.

bench.py times them, tests/golden/make_large_fixtures.py runs the CPU checker over them to
produce the committed per-frame digests (tests/golden/large_gops.json), and the `-m gpu`
tests and bench.py check the HIP path's output against those digests.

Every workload: bs 16, sr 16, intra_mode 0, nRefFrames 1, lambda 0.015, FME / fast_me off,
VBS off (the headline is VBS off).  Seeds per SURVEY.md §8(d): 0 for
configs 1-3, 1 for config 4 (the 120-frame GOP), 2 for config 5 (ROI + two-pass RC).

Variants of the benchmarked configs, each with its own per-frame digests (bench.py --config
NAME / --vbs / --me print parity.bit_exact for them):
  *_vbs          VBSEnable (the split decision of Encoder.py:512-578), lambda 0.015;
  1080p_fme      FMEEnable (half-pel search, Encoder.py:388-406, 697-705), 10 frames;
  1080p_fast     fast_me under ParallelMode 0 (the serial predictor chain, :719-742), 10 frames;
  1080p_fastpar  fast_me under ParallelMode 2 (predictor (0, 0, 0) per block, :587-676);
  4k_lowtex, 4k_noise  the headline on worst-case content for the exact SEA search
                 (synth.py `content`): the reference's scan costs the same on any content.
Keys: vbs (bool), me ("full" | "fme" | "fast" | "fastpar"), content (synth.py CONTENTS).
"""
from __future__ import annotations

# QP-rate table of tests/golden/rc_schedule.json scaled to 4K rows (x 11): the reference's
# get_appropriate_Qp_value (Encoder.py:1576-1580) then picks mid-range QPs at 50 mbps.
RC_TABLES = [[v * 11 for v in (9000, 6000, 4000, 2600, 1700, 1100, 700, 450, 300, 200)],
             [v * 11 for v in (7000, 4500, 3000, 2000, 1300, 850, 550, 350, 230, 150)]]

WORKLOADS = {
    # configs[1]: 1920x1080 source frames, pad_hw to 1920x1088 (Encoder.py:140-155, :1833)
    "1080p": dict(workload="1080p 30-frame I+P GOP (configs[1], 1920x1088 internal)", h=1080, w=1920, frames=30,
                  intra_dur=30, qp=4, seed=0),
    # configs[2]: the single-GPU 4K GOP
    "4k": dict(workload="4K 30-frame I+P GOP (configs[2])", h=2160, w=3840, frames=30, intra_dur=30, qp=4, seed=0),
    # configs[3]: one 120-frame GOP, sharded across the ranks
    "4k120": dict(workload="4K 120-frame I+P GOP (configs[3])", h=2160, w=3840, frames=120, intra_dur=120, qp=4,
                  seed=1),
    # configs[4]: ROI + two-pass RC (RCFlag 3, build extension): a centred ROI
    # rectangle at -2 QP, 50 mbps against RC_TABLES
    "4k_rc2pass": dict(workload="4K 30-frame ROI + two-pass RC GOP (configs[4])", h=2160, w=3840, frames=30,
                       intra_dur=30, qp=4, seed=2, rc=3, target="50 mbps", roi=[(1280, 720, 2560, 1440, -2)]),
    # variants (the SURVEY's VBS-on variant of the headline, the other ME modes, content)
    "4k_vbs": dict(workload="4K 30-frame I+P GOP, VBSEnable (configs[2] VBS-on variant)", h=2160, w=3840, frames=30,
                   intra_dur=30, qp=4, seed=0, vbs=True),
    "1080p_vbs": dict(workload="1080p 30-frame I+P GOP, VBSEnable (configs[1] VBS-on variant)", h=1080, w=1920,
                      frames=30, intra_dur=30, qp=4, seed=0, vbs=True),
    "1080p_fme": dict(workload="1080p 10-frame I+P GOP, FMEEnable (half-pel ME)", h=1080, w=1920, frames=10,
                      intra_dur=10, qp=4, seed=0, me="fme"),
    "1080p_fast": dict(workload="1080p 10-frame I+P GOP, fast_me, ParallelMode 0 (predictor chain)", h=1080,
                       w=1920, frames=10, intra_dur=10, qp=4, seed=0, me="fast"),
    "1080p_fastpar": dict(workload="1080p 10-frame I+P GOP, fast_me, ParallelMode 2", h=1080, w=1920, frames=10,
                          intra_dur=10, qp=4, seed=0, me="fastpar"),
    "4k_lowtex": dict(workload="4K 30-frame I+P GOP on low-texture content (32x32 flat cells, +-1 noise)", h=2160,
                      w=3840, frames=30, intra_dur=30, qp=4, seed=0, content="lowtex"),
    "4k_noise": dict(workload="4K 30-frame I+P GOP on noise-only content (128 +- 8 per pixel)", h=2160, w=3840,
                     frames=30, intra_dur=30, qp=4, seed=0, content="noise"),
}

# Y_Video_codec keyword arguments of each ME mode (Encoder.py:24)
ME_KW = {"full": {}, "fme": dict(FMEEnable=True), "fast": dict(fast_me=True),
         "fastpar": dict(fast_me=True, ParallelMode=2), "fast_fme": dict(fast_me=True, FMEEnable=True)}


def variant_name(name: str, vbs: bool = False, me: str = "full") -> str:
    """The workload key of `name` with VBSEnable / an ME mode applied (bench.py --vbs / --me),
    e.g. ("4k", vbs=True) -> "4k_vbs"; the name itself if no such variant exists."""
    base = WORKLOADS[name]
    vbs, me = vbs or base.get("vbs", False), me if me != "full" else base.get("me", "full")
    for k, v in WORKLOADS.items():
        if (v["h"], v["w"], v["seed"], v.get("rc"), v.get("content", "bench")) == \
                (base["h"], base["w"], base["seed"], base.get("rc"), base.get("content", "bench")) and \
                v.get("vbs", False) == vbs and v.get("me", "full") == me and \
                (v["frames"] == base["frames"] or me != "full" or vbs != base.get("vbs", False)):
            return k
    return name


def padded(n: int, bs: int = 16) -> int:
    return -(-n // bs) * bs


def roi_offsets(roi, h: int, w: int, bs: int):
    """ROI as int32 [nb] per-block QP offsets in raster order (or None): `roi` is a
    [ceil(h/bs), ceil(w/bs)] array, or rectangles (x0, y0, x1, y1, offset) in pixels -- a
    block takes the offset of the last rectangle holding its centre."""
    import numpy as np
    if roi is None:
        return None
    nby, nbx = padded(h, bs) // bs, padded(w, bs) // bs
    a = np.asarray(roi)
    if a.ndim == 2 and a.shape == (nby, nbx):
        return a.astype(np.int32).reshape(-1)
    out = np.zeros((nby, nbx), np.int32)
    cy = np.arange(nby)[:, None] * bs + bs / 2
    cx = np.arange(nbx)[None, :] * bs + bs / 2
    for x0, y0, x1, y1, off in roi:
        out[(cy >= y0) & (cy < y1) & (cx >= x0) & (cx < x1)] = int(off)
    return out.reshape(-1)
