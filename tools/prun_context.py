"""Why the P-run is slower inside the GOP step than replayed back to back: the same
persistent launch (29 P-frames of the bench's 4K GOP) timed with HIP events on its stream,
(a) back to back, (b) after the I-frame kernels as in a step, (c) after an idle gap of the
I-frame's length (host sleep), (d) after a short dummy kernel."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from streamoptima_amd.engine import Engine, alloc_planes
    from streamoptima_amd.synth import synth_sequence_torch
    dev = torch.device("cuda:0")
    h, w, f = 2160, 3840, 30
    eng = Engine(h, w, 16, 16, False, 0.015, dev)
    fr = alloc_planes(f, h, w, dev)
    fr.copy_(synth_sequence_torch(f, h, w, seed=0, device=dev))
    i0 = eng.encode_i(fr[0], 4)
    outs = [eng.new_symbols(1) for _ in range(f - 1)]
    curs = [fr[i] for i in range(1, f)]
    st = torch.cuda.current_stream(dev)

    def prun():
        eng.encode_p_run(curs, i0.recon, 4, outs)

    def timed(pre, reps=12):
        ts = []
        for _ in range(reps):
            pre()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            prun()
            b.record(st)
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        ts = sorted(ts[2:])
        return [round(ts[0], 1), round(ts[len(ts) // 2], 1)]
    out = {"back_to_back": timed(lambda: prun()),
           "after_iframe": timed(lambda: eng.encode_i(fr[0], 4, out=i0)),
           "after_idle_80us": timed(lambda: time.sleep(80e-6)),
           "after_sum_rows": timed(lambda: eng.sum_rows([o.sse for o in outs]))}
    eng.check_run()
    print(json.dumps({"p_run_us_min_median": out}))


if __name__ == "__main__":
    main()
