"""Per-GOP kernel timeline from a rocprofv3 --kernel-trace CSV: for the last N GOPs (a GOP starts
at an intra_tq_kernel launch), every kernel's duration and the gap before it, in microseconds.
    python tools/gop_timeline.py gpurun_out/.../run_kernel_trace.csv [N]"""
import csv
import re
import sys


def short(name: str) -> str:
    m = re.search(r"(so::)?([A-Za-z_0-9]+)(<[^()]*>)?\(", name)
    return (m.group(2) + (m.group(3) or "")) if m else name[:40]


def main(path: str, n: int = 2) -> None:
    rows = list(csv.DictReader(open(path)))
    ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows))
    starts = [i for i, e in enumerate(ev) if e[2].startswith("intra_tq_kernel")]
    for k, i0 in enumerate(starts[-n - 1:-1] if len(starts) > n else starts[:-1]):
        nxt = starts[starts.index(i0) + 1]
        t0, prev_end = ev[i0][0], ev[i0][0]
        print(f"GOP at index {i0}: {(ev[nxt - 1][1] - t0) / 1e3:.1f} us to the last kernel before the next GOP")
        for s, e, nm in ev[i0:nxt]:
            print(f"  +{(s - t0) / 1e3:8.1f}  gap {(s - prev_end) / 1e3:6.1f}  dur {(e - s) / 1e3:8.1f}  {nm}")
            prev_end = e


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2)
