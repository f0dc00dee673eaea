"""tests/mp_util.py on the CPU (no GPU touched): rank r goes to device r % device_count -- one rank per
GPU on a node, every rank on device 0 of a one-GPU box, where more than two ranks get one hardware
queue each -- and `collect` fails as soon as a rank process dies without a result."""
import multiprocessing as mp
import os

import pytest
import torch

import mp_util


@pytest.mark.parametrize("ndev,n", [(8, 8), (8, 2), (1, 2), (1, 4), (2, 4)])
def test_place_rank(monkeypatch, ndev, n):
    placed = []
    monkeypatch.setattr(torch.cuda, "device_count", lambda: ndev)
    monkeypatch.setattr(torch.cuda, "set_device", lambda d: placed.append(d))
    monkeypatch.delenv("GPU_MAX_HW_QUEUES", raising=False)
    out = [mp_util.place_rank(r, n) for r in range(n)]
    assert placed == [r % ndev for r in range(n)]
    assert all(shared == (ndev < n) for _, shared in out)
    assert (os.environ.get("GPU_MAX_HW_QUEUES") == "1") == (ndev < n and n > 2)
    if ndev >= n:
        assert len(set(placed)) == n  # a rank per GPU


def _dies(code):
    os._exit(code)


def test_collect_fails_fast_on_a_dead_rank():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dies, args=(3,))]
    procs[0].start()
    with pytest.raises(pytest.fail.Exception, match="died without a result"):
        mp_util.collect(procs, q, 1, timeout=60)
