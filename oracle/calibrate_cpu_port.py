#!/usr/bin/env python
"""Calibrate the CPU baseline (oracle/ref_numpy.py) against the reference itself.

    python oracle/calibrate_cpu_port.py [--rows 3]

Development container only (needs /root/reference).  TEST INFRASTRUCTURE.  It imports the
reference the way tests/golden/make_golden.py does (skimage stub, Agg backend), builds a
3840-wide band of `rows` block rows of the synthetic sequence, and times on IDENTICAL
inputs:
  * the reference's complete_inter_flow (Encoder.py:1644-1709) on the band vs
    ref_numpy.inter_rows over the same rows (same candidates, bounds, transforms, tokens);
  * the reference's complete_intra_flow (Encoder.py:1582-1642; canvas patched to the band
    size) vs ref_numpy.intra_rows;
and writes profiles/cpu_port_calibration.json with both times, the ratio (BASELINE.md §3:
the port must be within +-20 % of the reference) and the token counts of both, which must be
equal.  bench.py's cpu_baseline quotes this record.
"""
from __future__ import annotations

import argparse
import contextlib
import importlib.util
import io
import json
import os
import platform
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[0] = ROOT   # not oracle/ itself: oracle/oracle.py would shadow the package


def _make_golden():
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(ROOT, "tests", "golden", "make_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def main():
    from oracle.ref_numpy import inter_rows, intra_rows
    from streamoptima_amd.synth import synth_sequence
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=3)
    a = ap.parse_args()
    mg = _make_golden()
    Enc, _ = mg.import_reference()
    h, w = 16 * a.rows, 3840
    seq = synth_sequence(2, h, w, seed=0)
    cur, ref = seq[1], seq[0]
    out = {"host": cpu_model(), "cores": 1, "band": f"{w}x{h} ({a.rows} block rows, {a.rows * w // 16} blocks)"}
    with tempfile.TemporaryDirectory() as tmp:
        os.makedirs(os.path.join(tmp, "files"))
        os.makedirs(os.path.join(tmp, "yuv"))
        old = os.getcwd()
        os.chdir(tmp)
        try:
            enc = Enc.Y_Video_codec(h, w, 2, 16, 16, 4, 2, 0, 0.015, False, y_only_frame_arr=seq)
            padded = enc.pad_hw(cur, 16, 128)
            with contextlib.redirect_stdout(io.StringIO()):
                t0 = time.perf_counter()
                r = enc.complete_inter_flow(padded, [ref], 16, 16)
                t_ref_p = time.perf_counter() - t0
            ref_tok_p = int(r[5])
            t0 = time.perf_counter()
            port_tok_p, _ = inter_rows(padded, ref, range(a.rows))
            t_port_p = time.perf_counter() - t0
            with mg.canvas_patch(Enc, h, w), contextlib.redirect_stdout(io.StringIO()):
                enc.set_Qp(4)
                t0 = time.perf_counter()
                ri = enc.complete_intra_flow(padded, 0, 16, 16)
                t_ref_i = time.perf_counter() - t0
            ref_tok_i = int(ri[6])
            t0 = time.perf_counter()
            port_tok_i = intra_rows(padded, range(a.rows))
            t_port_i = time.perf_counter() - t0
        finally:
            os.chdir(old)
    px = h * w
    out.update({
        "p_frame": {"reference_s": round(t_ref_p, 3), "port_s": round(t_port_p, 3),
                    "port_over_reference_time": round(t_port_p / t_ref_p, 4),
                    "reference_mpx_s": round(px / t_ref_p / 1e6, 5), "port_mpx_s": round(px / t_port_p / 1e6, 5),
                    "tokens_reference": ref_tok_p, "tokens_port": port_tok_p},
        "i_frame": {"reference_s": round(t_ref_i, 3), "port_s": round(t_port_i, 3),
                    "port_over_reference_time": round(t_port_i / t_ref_i, 4),
                    "tokens_reference": ref_tok_i, "tokens_port": port_tok_i},
    })
    out["within_20pct"] = bool(abs(out["p_frame"]["port_over_reference_time"] - 1) <= 0.2)
    out["tokens_equal"] = ref_tok_p == port_tok_p and ref_tok_i == port_tok_i
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "cpu_port_calibration.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
