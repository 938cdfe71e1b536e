"""BASELINE.md §3's full-frame CPU timing: the numpy port of the reference loops
(oracle/ref_numpy.py, calibrated against the reference: profiles/cpu_port_calibration.json)
over EVERY block row of one 4K P-frame and one 4K I-frame of the bench workload, serially, on
the host it runs on (run once on the GPU box; bench.py's cpu_baseline extrapolates 8 rows).
TEST / MEASUREMENT INFRASTRUCTURE.
    python tools/cpu_full_frame.py > profiles/r03/cpu_full_frame.json"""
import json
import os
import platform
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from oracle.ref_numpy import inter_rows, intra_rows
    from streamoptima_amd.synth import synth_sequence
    h, w = 2160, 3840
    seq = synth_sequence(2, h, w, seed=0)
    cur, ref = seq[1].astype(np.float64), seq[0]
    rows = range(h // 16)
    t0 = time.perf_counter()
    tok_p, _ = inter_rows(cur, ref, rows, qp=4)
    tp = time.perf_counter() - t0
    t0 = time.perf_counter()
    tok_i = intra_rows(cur, rows, qp=4)
    ti = time.perf_counter() - t0
    model = next((l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")),
                 platform.processor())
    gop = tp * 29 + ti
    print(json.dumps({"what": "numpy port of Encoder.py's loops, one full 3840x2160 frame of each type, serial",
                      "p_frame_s": round(tp, 2), "i_frame_s": round(ti, 2), "p_frame_mpx_s": round(h * w / tp / 1e6, 5),
                      "gop30_s_extrapolated": round(gop, 1), "gop30_mpx_s": round(30 * h * w / gop / 1e6, 5),
                      "tokens_p": int(tok_p), "tokens_i": int(tok_i), "cores": 1, "host": model,
                      "os_cpu_count": os.cpu_count()}), flush=True)


if __name__ == "__main__":
    main()
