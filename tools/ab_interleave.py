"""A/B of P-run per-frame time, variants interleaved round by round (each run a fresh process),
so a box's clock drift over the minutes of an A/B lands on every variant alike:
    python tools/ab_interleave.py --rounds 3 default tools/_ab/a.so SO_RUN_PER_CU=2 ...
Prints one JSON line per variant: per size, the min over rounds of each run's min and the median
of the runs' medians (us per frame)."""
import argparse
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ab_runs import CHILD  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ab_guard import require_ab_build  # noqa: E402
require_ab_build()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    res = {v: [] for v in a.variants}
    for rd in range(a.rounds):
        for v in (a.variants if rd % 2 == 0 else a.variants[::-1]):
            env = dict(os.environ)
            for part in v.split(":"):          # lib.so, ENV=VAL, or lib.so:ENV=VAL[:ENV=VAL]
                if "=" in part:
                    k, val = part.split("=", 1)
                    env[k] = val
                elif part != "default":
                    env["SO_LIB_PATH"] = part
            r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
            line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            if not line:
                print(json.dumps({"variant": v, "error": r.stderr[-800:]}), flush=True)
                sys.exit(1)
            res[v].append(json.loads(line[-1]))
            print(json.dumps({"round": rd, "variant": v, "us_per_frame_min_median": res[v][-1]}), flush=True)
    for v, runs in res.items():
        out = {}
        for size in runs[0]:
            mins = sorted(r[size][0] for r in runs)
            meds = sorted(r[size][1] for r in runs)
            out[size] = [mins[0], meds[len(meds) // 2]]
        print(json.dumps({"variant": v, "summary_min_median": out}), flush=True)


if __name__ == "__main__":
    main()
