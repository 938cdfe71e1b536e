"""The frame pipeline's host-side plan (pipeline.fpipe_plan) on CPU: every P-frame's
reference lands in exactly the slot its encoder reads, and a tile-level simulation of the N
persistent launches (frame-major task order, a few resident workgroups per rank, 3x3 tile
dependencies on the previous frame's rank) always drains -- no deadlock for any world size."""
import itertools

import pytest

from streamoptima_amd.pipeline import fpipe_plan


@pytest.mark.parametrize("world", [2, 3, 4, 5, 8])
@pytest.mark.parametrize("nframes", [1, 2, 7, 30, 120])
def test_reference_slots_match(world, nframes):
    plans = [fpipe_plan(world, g, nframes) for g in range(world)]
    assert sorted(itertools.chain.from_iterable(p["frames"] for p in plans)) == list(range(nframes))
    for g, p in enumerate(plans):
        for i, k in enumerate(p["run"]):
            slot = p["slot0"] + i                      # the slot this frame's launch reads
            assert slot == (k - g) // world and slot < p["nslots"]
            prod = (k - 1) % world                     # who encodes frame k-1 ...
            pp = plans[prod]
            pslot = ((k - 1) - prod) // world          # ... in its slot ...
            push = 0 if k - 1 == 0 else pslot + pp["peer_slot_off"]   # ... and where it pushes it
            assert (prod + 1) % world == g and push == slot
            assert push < plans[(prod + 1) % world]["nslots"]


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
