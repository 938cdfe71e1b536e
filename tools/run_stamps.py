"""Where a persistent P-frame run's time goes, per tile task (p_run_kernel, SO_STAMPS build).

    python -m streamoptima_amd.build --out tools/_ab/stamps.so -D SO_STAMPS
    SO_LIB_PATH=tools/_ab/stamps.so python tools/run_stamps.py [--heights 272,1088,2160] [--width 3840]

For every (frame, tile) task: the dequeue, wait start / end and done times (s_memrealtime,
100 MHz, one clock for the whole chip) and the phase cycles inside the tile (s_memtime of
its CU): current-tile staging, dependency wait + acquire, window staging, 4x4 byte sums,
search, transforms + stores.  The hand-off latency of a dependency is the consumer's wait
end minus the last of its 3x3 producers' done times.  The chain step (frame-to-frame time of
one tile position) is what sets the per-frame time once a frame has fewer tiles than the
chip has resident workgroups (4K stripes at N ranks, 1080p).
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def analyse(rec, nframes, tiles_x, ntr):
    ntiles = tiles_x * ntr
    r = rec.reshape(nframes, ntiles, 16).astype(np.int64)
    rt = lambda k: r[:, :, k].astype(np.float64) * 0.01    # noqa: E731  us (100 MHz)
    deq, w0, w1, done = rt(8), rt(9), rt(10), rt(11)
    cyc = lambda a, b: (r[1:, :, b] - r[1:, :, a]).astype(np.float64)  # noqa: E731
    out = {}
    # hand-off: wait end - last producer done (frames >= 1)
    lat, step = [], []
    for f in range(1, nframes):
        for t in range(ntiles):
            ty, tx = divmod(t, tiles_x)
            prod = [done[f - 1, ny * tiles_x + nx] for ny in range(ty - 1, ty + 2) for nx in range(tx - 1, tx + 2)
                    if 0 <= ny < ntr and 0 <= nx < tiles_x]
            last = max(prod)
            if w1[f, t] >= last:         # waited for its producers (not already done on arrival)
                lat.append(w1[f, t] - last)
            step.append(done[f, t] - done[f - 1, t])
    t0 = deq.min()
    out["span_us"] = round(done.max() - t0, 2)
    out["per_frame_us"] = round((done.max() - t0) / nframes, 2)
    q = lambda a: [round(float(np.percentile(a, p)), 2) for p in (10, 50, 90)]  # noqa: E731
    out["handoff_us_p10_50_90"] = q(np.array(lat)) if lat else None
    out["tasks_that_waited"] = len(lat)
    out["chain_step_us_p10_50_90"] = q(np.array(step))
    out["tile_done_minus_wait_end_us"] = q((done[1:] - w1[1:]).ravel())
    out["wait_us"] = q((w1[1:] - w0[1:]).ravel())
    out["dequeue_to_wait_us"] = q((w0[1:] - deq[1:]).ravel())
    # phases in shader cycles (memtime): [1] start, [2] after wait+acquire+barrier, [3] window,
    # [4] byte sums, [5] search done, [13] transforms + stores + flag
    out["cycles_p50"] = {
        "stage_cur_wait": float(np.median(cyc(1, 2))), "window": float(np.median(cyc(2, 3))),
        "b4": float(np.median(cyc(3, 4))), "search": float(np.median(cyc(4, 5))),
        "decode": float(np.median(cyc(5, 6))), "tq_wave0": float(np.median(cyc(6, 7))),
        "store_drain_wave0": float(np.median(cyc(7, 14))), "barrier_flag": float(np.median(cyc(14, 13))),
        "tq_store_flag": float(np.median(cyc(5, 13)))}
    # the search phase's spread: a tile whose wave holds a dense-fallback block keeps its other
    # waves at the barrier (mean vs median, p90 / p99)
    sc = cyc(4, 5).ravel()
    out["search_cycles_mean_p50_p90_p99"] = [round(float(sc.mean())), round(float(np.median(sc))),
                                            round(float(np.percentile(sc, 90))), round(float(np.percentile(sc, 99)))]
    tot = cyc(1, 13).ravel()
    out["tile_cycles_mean_p50_p90"] = [round(float(tot.mean())), round(float(np.median(tot))),
                                       round(float(np.percentile(tot, 90)))]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--heights", default="272,1088,2160")
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--frames", type=int, default=24)
    ap.add_argument("--vbs", action="store_true", help="VBSEnable (p_run_kernel<8, 0, true>)")
    a = ap.parse_args()
    from streamoptima_amd import _lib
    from streamoptima_amd.engine import Engine, alloc_planes
    from streamoptima_amd.synth import synth_sequence_torch
    dev = torch.device("cuda:0")
    lib = _lib.load()
    lib.so_debug_set_run_stamps.argtypes = [ctypes.c_void_p]
    res = {}
    for h in [int(x) for x in a.heights.split(",")]:
        w = a.width
        eng = Engine(h, w, 16, 16, a.vbs, 0.015, dev)
        nf = a.frames + 1
        fr = alloc_planes(nf, h, w, dev)
        fr.copy_(synth_sequence_torch(nf, h, w, seed=0, device=dev))
        i0 = eng.encode_i(fr[0], 4)
        outs = [eng.new_symbols(1) for _ in range(nf - 1)]
        curs = [fr[i] for i in range(1, nf)]
        tiles_x, ntr = -(-(w // 16) // 8), -(-(h // 16) // 2)
        stamps = torch.zeros(((nf - 1) * tiles_x * ntr, 16), dtype=torch.int64, device=dev)
        eng.encode_p_run(curs, i0.recon, 4, outs)                 # warm
        assert lib.so_debug_set_run_stamps(stamps.data_ptr()) == 0
        eng.encode_p_run(curs, i0.recon, 4, outs)
        torch.cuda.synchronize()
        assert lib.so_debug_set_run_stamps(None) == 0
        eng.check_run()
        res[h] = analyse(stamps.cpu().numpy(), nf - 1, tiles_x, ntr)
        print(f"H={h} W={w}:", json.dumps(res[h]), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
