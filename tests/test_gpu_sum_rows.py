"""so_sum_i32_rows (Engine.sum_rows): the per-frame SSE sum of encode_device, one launch --
exact int64 sums for aligned and misaligned rows, lengths around the vector width, more
rows than one launch takes."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_sum_rows_exact(gpu):
    from streamoptima_amd.engine import Engine
    e = Engine(64, 128, 16, 16, False, 0.015, gpu)
    g = torch.Generator(device=gpu).manual_seed(7)
    for n in (1, 5, 7, 2160, 32400, 32401, 100003):
        rows = [torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device=gpu, generator=g) for _ in range(70)]
        want = torch.stack([r.to(torch.int64).sum() for r in rows])
        assert torch.equal(e.sum_rows(rows), want), n
        mis = [torch.randint(-1000, 1000, (n + 1,), dtype=torch.int32, device=gpu, generator=g)[1:] for _ in range(3)]
        assert torch.equal(e.sum_rows(mis), torch.stack([r.to(torch.int64).sum() for r in mis])), n
