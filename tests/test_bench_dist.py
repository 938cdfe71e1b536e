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
