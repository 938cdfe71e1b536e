"""Phase attribution of p_run_kernel (the headline's persistent fused search + transform
launch): the 4K P-run of the bench GOP (29 frames) timed with HIP events, for the library
named by SO_LIB_PATH -- the product build, or an A/B build with -DSO_PROF_PHASE=1 (transforms
compiled out) / =2 (search compiled out: every block at mv (0, 0)).  Run under
`rocprofv3 --pmc ...` for the per-phase instruction counts (tools/gpu_r03c.sh).
    python tools/prun_phase.py [--reps N]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--h", type=int, default=2160)
    ap.add_argument("--w", type=int, default=3840)
    ap.add_argument("--vbs", action="store_true", help="VBSEnable (p_run_kernel<8, 0, true>)")
    a = ap.parse_args()
    from streamoptima_amd.engine import Engine, alloc_planes
    from streamoptima_amd.synth import synth_sequence_torch
    dev = torch.device("cuda:0")
    f = 30
    eng = Engine(a.h, a.w, 16, 16, a.vbs, 0.015, dev)
    fr = alloc_planes(f, a.h, a.w, dev)
    fr.copy_(synth_sequence_torch(f, a.h, a.w, seed=0, device=dev))
    i0 = eng.encode_i(fr[0], 4)
    outs = [eng.new_symbols(1) for _ in range(f - 1)]
    curs = [fr[i] for i in range(1, f)]
    for _ in range(3):
        eng.encode_p_run(curs, i0.recon, 4, outs)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(a.reps):
        e0.record()
        eng.encode_p_run(curs, i0.recon, 4, outs)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    eng.check_run()
    ts.sort()
    print(json.dumps({"lib": os.environ.get("SO_LIB_PATH", "default"), "vbs": a.vbs, "frames": f - 1,
                      "launch_us_min": round(ts[0], 1), "launch_us_median": round(ts[len(ts) // 2], 1),
                      "us_per_frame_median": round(ts[len(ts) // 2] / (f - 1), 2)}), flush=True)


if __name__ == "__main__":
    main()
