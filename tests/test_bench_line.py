"""The driver parses bench.py's last stdout line: it must stay valid JSON of bounded size
(round 5's 22.9 KB line went unparsed; bench.py LINE_MAX_BYTES), keep the contract's keys
(value, roofline, cpu_baseline) and every record's numbers, and be the last line printed."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
FULL = os.path.join(ROOT, "tests", "fixtures", "bench_line_r05_full.json")


def _full():
    with open(FULL) as fh:
        return json.load(fh)


def test_compact_line_of_round5_full_line_is_bounded_and_complete():
    import bench
    full = _full()
    assert len(json.dumps(full)) > 20000          # the line the driver could not parse
    line = bench.compact_line(full)
    s = json.dumps(line)
    assert len(s) <= bench.LINE_MAX_BYTES
    assert json.loads(s) == line
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert line[k] == full[k] if k != "config" else line[k]["workload"] == full[k]["workload"]
    rl = line["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert rl[k] == full["roofline"][k]
    assert rl["valu_profile"]["valu_busy_frac"] == full["roofline"]["valu"]["valu_busy_frac"]
    cpu = line["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind"):
        assert cpu[k] == full["cpu_baseline"][k]
    assert cpu["sample"].startswith("8 block rows")
    assert line["section4_region"]["value"] == full["section4_region"]["value"]
    assert set(line["records"]) == set(full["records"])
    for name, r in full["records"].items():
        c = line["records"][name]
        assert c["ms_per_step"] == r["ms_per_step"] and c["value"] == r["value"]
        assert c["parity"]["bit_exact"] is True
        if "roofline" in r:
            assert c["roofline"]["frac"] == r["roofline"]["frac"]
            assert c["roofline"]["traffic"] == r["roofline"]["traffic"]
    assert "algorithmic_bytes" in line["defs"] and "valu_profile" in line["defs"]


def test_compact_line_stays_bounded_when_every_record_fails():
    """Error entries and wait-timeout records must not push the line past the bound."""
    import bench
    full = _full()
    for name in list(full["records"]):
        full["records"][name] = {"error": "RuntimeError: " + "x" * 300}
    for i in range(20):
        full["records"][f"extra{i}"] = {"value": 1.0, "ms_per_step": 1.0, "workload": "w" * 200,
                                        "wait_health": {"timeouts": 3, "records": [{"task": 35, "frame": 0}] * 4}}
    line = bench.compact_line(full)
    assert len(json.dumps(line)) <= bench.LINE_MAX_BYTES


def test_cpu_plumbing_line_is_last_bounded_json(tmp_path):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    detail = tmp_path / "detail.json"
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu-plumbing", "--frames", "2",
                          "--steps", "1", "--warmup", "0", "--detail-out", str(detail)],
                         env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    last = out.stdout.rstrip("\n").splitlines()[-1]
    import bench
    assert len(last.encode()) <= bench.LINE_MAX_BYTES
    line = json.loads(last)
    assert line["value"] > 0 and line["n_gpus"] == 1 and "defs" in line
    assert json.loads(detail.read_text())["value"] == line["value"]
