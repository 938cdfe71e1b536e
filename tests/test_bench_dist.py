"""bench.py's multi-rank plumbing on CPU (gloo, world size 2): dist_setup from the torchrun
environment, the timing barrier and the max-over-ranks reduction of the step time that
makes the JSON line's whole-job value (the driver runs the same code over RCCL)."""
import os
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rank(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    import bench
    import torch.distributed as dist
    w, r, loc = bench.dist_setup(backend="gloo")
    bench.barrier(w)
    m = bench.max_over_ranks(1.0 + r, w)
    q.put((r, w, loc, m))
    dist.destroy_process_group()


def test_bench_max_over_ranks_gloo():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out == [(0, 2, 0, 2.0), (1, 2, 1, 2.0)]


def test_bench_single_rank_defaults():
    sys.path.insert(0, ROOT)
    import bench
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        os.environ.pop(k, None)
    assert bench.dist_setup(backend="gloo") == (1, 0, 0)
    assert bench.max_over_ranks(3.5, 1) == 3.5


def test_bench_gpus_flag_launches_ranks_cpu_plumbing():
    """`bench.py --gpus 2` with no torchrun environment re-launches itself as 2 ranks
    (torch.distributed.run) and rank 0 prints n_gpus 2 for configs[3] (one 4K GOP sharded
    over the ranks, strong scaling).  --cpu-plumbing swaps the HIP engine for a trivial CPU
    stand-in (gloo), so this runs without a GPU; --frames keeps it short."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu-plumbing", "--gpus", "2",
                          "--frames", "3", "--steps", "1", "--warmup", "1"], env=env, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads([x for x in out.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert line["config"]["name"] == "4k120" and "configs[3]" in line["config"]["workload"]
    assert line["config"]["parallelism"].startswith("stripe x2")


def test_bench_gpus_mismatch_is_an_error():
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu-plumbing", "--gpus", "2"], env=env,
                         capture_output=True, text=True, timeout=120)
    assert out.returncode != 0 and "WORLD_SIZE 1" in out.stderr


def test_bench_secondary_failure_keeps_the_headline_line():
    """A failing secondary measurement (a record, the PCIe leg, the CPU baseline) is recorded in
    the line as {"error": ...} and named in `failed`; the headline line is still printed, and the
    exit status is nonzero so the failure stays visible (no retry, no silent pass)."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu-plumbing", "--frames", "2",
                          "--steps", "1", "--warmup", "0", "--inject-failure", "records.1080p_x2gop"], env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode != 0
    line = json.loads([x for x in out.stdout.splitlines() if x.startswith("{")][-1])
    assert line["value"] > 0 and line["failed"] == ["records.1080p_x2gop"]
    assert "injected" in line["records"]["records.1080p_x2gop"]["error"] or \
        "--inject-failure" in line["records"]["records.1080p_x2gop"]["error"]
    assert "measurement(s) failed or degraded" in out.stderr


def test_bench_multi_gpu_fallback_is_loud():
    """A multi-GPU path whose self-check fails is replaced by a fallback (frame pipeline ->
    stripes -> RCCL all_gather), and that must never pass silently for the default path's time:
    the line still prints, names the degradation under `degraded` and `failed`, and the exit
    status is nonzero.  --inject-failure fpipe_selfcheck makes the self-check fail (on the GPU
    box it forces the real self-check's verdict; here the CPU stand-in takes the same branch)."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu-plumbing", "--gpus", "2",
                          "--frames", "3", "--steps", "1", "--warmup", "0", "--inject-failure", "fpipe_selfcheck"],
                         env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode != 0
    line = json.loads([x for x in out.stdout.splitlines() if x.startswith("{")][-1])
    assert line["value"] > 0 and line["n_gpus"] == 2
    assert line["failed"] == ["fpipe_selfcheck"]
    assert line["degraded"][0]["what"] == "fpipe_selfcheck" and "stripes" in line["degraded"][0]["timed_instead"]
    assert "degraded" in out.stderr
