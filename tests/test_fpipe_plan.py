"""The frame pipeline's host-side plan (pipeline.fpipe_plan) on CPU: every P-frame's
reference lands in exactly the slot its encoder reads, and a tile-level simulation of the N
persistent launches (frame-major task order, a few resident workgroups per rank, 3x3 tile
dependencies on the previous frame's rank) always drains -- no deadlock for any world size."""
import itertools

import pytest

from streamoptima_amd.pipeline import fpipe_plan, fpipe_rank_of


@pytest.mark.parametrize("world", [2, 3, 4, 5, 8])
@pytest.mark.parametrize("nframes", [1, 2, 7, 30, 120])
def test_reference_slots_match(world, nframes):
    plans = [fpipe_plan(world, g, nframes) for g in range(world)]
    assert sorted(itertools.chain.from_iterable(p["frames"] for p in plans)) == list(range(nframes))
    owner = {k: g for g, p in enumerate(plans) for k in p["frames"]}
    assert all(owner[k] == fpipe_rank_of(world, k) for k in range(nframes))
    for g, p in enumerate(plans):
        assert p["frames"] == sorted(p["frames"])
        for i, k in enumerate(p["run"]):
            slot = p["slot0"] + i                      # the slot this frame's launch reads
            assert slot == k // world and slot < p["nslots"]
            # where this frame's reconstruction goes: the rank of frame k + 1, its slot
            code = p["push"][i]
            if k == nframes - 1:                       # nothing follows the GOP's last frame
                assert code == -1
                continue
            dst = (g + 1) % world if code % 2 == 0 else (g - 1) % world
            assert dst == fpipe_rank_of(world, k + 1) and code // 2 == (k + 1) // world
            assert code // 2 < plans[dst]["nslots"]
    if world > 2 and nframes >= 2 * world:   # both ring directions carry frames
        codes = [c % 2 for p in plans for c in p["push"] if c >= 0]
        assert 0 < sum(codes) < len(codes)


def _simulate(world, nframes, tiles_x, tiles_y, wgs):
    """Discrete steps: each rank's workgroups take (frame, tile) tasks in frame-major order and
    finish a task one step after all 3x3 tiles of the previous frame are done."""
    plans = [fpipe_plan(world, g, nframes) for g in range(world)]
    queues = [[(k, t) for k in p["run"] for t in range(tiles_x * tiles_y)] for p in plans]
    done = {(0, t) for t in range(tiles_x * tiles_y)}           # the I-frame, pushed before the runs
    held = [[None] * wgs for _ in range(world)]
    for step in range(100000):
        progress = False
        for g in range(world):
            for w in range(wgs):
                if held[g][w] is None and queues[g]:
                    held[g][w] = queues[g].pop(0)
                    progress = True
                task = held[g][w]
                if task is None:
                    continue
                k, t = task
                tx, ty = t % tiles_x, t // tiles_x
                deps = [(k - 1, ny * tiles_x + nx) for ny in range(ty - 1, ty + 2) for nx in range(tx - 1, tx + 2)
                        if 0 <= nx < tiles_x and 0 <= ny < tiles_y]
                if all(d in done for d in deps):
                    done.add(task)
                    held[g][w] = None
                    progress = True
        if all(not q for q in queues) and all(h is None for r in held for h in r):
            return step
        if not progress:
            raise AssertionError(f"deadlock at step {step}")
    raise AssertionError("did not drain")


@pytest.mark.parametrize("world,wgs", [(2, 1), (2, 3), (3, 2), (8, 1), (8, 4)])
def test_pipeline_drains(world, wgs):
    steps = _simulate(world, 17, tiles_x=4, tiles_y=3, wgs=wgs)
    assert steps > 0
