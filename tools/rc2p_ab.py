"""Per-GOP time of the configs[4] workload (4K ROI + two-pass RC) under environment
variants (SO_P2LAG=..., SO_PIPELINE=0), each in a fresh process:
    python tools/rc2p_ab.py SO_P2LAG=1 SO_P2LAG=68 SO_PIPELINE=0 SO_LIB_PATH=x.so,SO_P2LAG=68
(comma-joined settings form one variant; an SO_RUN_PROFILE library adds per-phase kcycles;
AB_FUSED=1 with SO_RUN_2PASS=1 runs the fused two-pass launch)"""
import json
import os
import subprocess
import sys

CHILD = r'''
import json, sys, time, torch
sys.path.insert(0, ".")
from bench import build_codec, make_frames, parse
from streamoptima_amd.workloads import WORKLOADS
dev = torch.device("cuda:0")
import os
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ab_guard import require_ab_build  # noqa: E402
require_ab_build()
cfg = dict(WORKLOADS[os.environ.get("AB_CFG", "4k_rc2pass")])
codec = build_codec(cfg, parse([]), dev)
if os.environ.get("AB_FUSED") == "1":   # both passes in one persistent launch (needs SO_RUN_2PASS=1)
    from streamoptima_amd import _lib
    _lib.set_option(_lib.OPT_RUN_2PASS_FUSED, 1)
fr = make_frames(cfg, dev, cfg["seed"])
ts, enq = [], []
for _ in range(6):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    codec.encode_device(fr, cfg["intra_dur"], check=False)
    enq.append(time.perf_counter() - t0)   # host time to enqueue the GOP
    torch.cuda.synchronize(); ts.append(time.perf_counter() - t0)
codec.engine().check_run()
ts = sorted(ts[1:])
out = {"ms_per_gop_min_median": [round(ts[0] * 1e3, 3), round(ts[len(ts) // 2] * 1e3, 3)],
       "host_enqueue_ms_median": round(sorted(enq[1:])[2] * 1e3, 3)}
ws = getattr(codec.engine(), "_run_ws", None)
if ws is not None and int(ws[48:53].sum()) > 0:   # SO_RUN_PROFILE library: kcycles per GOP
    out["kcycles_per_gop"] = {k: int(ws[48 + i]) // 6 for i, k in
                              enumerate(("pass1_task", "pass2_task", "pass2_row_wait", "ref_wait", "one_pass_task"))}
print(json.dumps(out))
'''


def main():
    for v in [""] + sys.argv[1:]:
        env = dict(os.environ)
        for kv in v.split(","):
            if kv:
                k, val = kv.split("=", 1)
                env[k] = val
        r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        print(json.dumps({"variant": v or "default", **(json.loads(line[-1]) if line else {"err": r.stderr[-400:]})}),
              flush=True)


if __name__ == "__main__":
    main()
