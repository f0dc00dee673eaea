"""tests/mp_util.py on the CPU (no GPU touched): rank r goes to device r % device_count -- one rank per
GPU on a node, every rank on device 0 of a one-GPU box, where more than two ranks get one hardware
queue each, decided from the parent's device count before HIP can start -- and `collect` fails as
soon as a rank process dies without a result."""
import multiprocessing as mp
import os

import pytest
import torch

import mp_util


@pytest.mark.parametrize("ndev,n", [(8, 8), (8, 2), (1, 2), (1, 4), (2, 4)])
def test_place_rank(monkeypatch, ndev, n):
    placed = []
    counted = []
    monkeypatch.setenv(mp_util.NDEV_ENV, str(ndev))
    # the exported count is used: device_count (which may start HIP) is never called
    monkeypatch.setattr(torch.cuda, "device_count", lambda: counted.append(1) or ndev)
    monkeypatch.setattr(torch.cuda, "set_device",
                        lambda d: placed.append((d, os.environ.get("GPU_MAX_HW_QUEUES"))))
    monkeypatch.delenv("GPU_MAX_HW_QUEUES", raising=False)
    out = [mp_util.place_rank(r, n) for r in range(n)]
    assert [d for d, _ in placed] == [r % ndev for r in range(n)]
    assert all(shared == (ndev < n) for _, shared in out)
    want = "1" if ndev < n and n > 2 else None
    assert all(q == want for _, q in placed)  # set before the first device call
    assert not counted
    if ndev >= n:
        assert len({d for d, _ in placed}) == n  # a rank per GPU


def test_place_rank_without_exported_count(monkeypatch):
    """No exported count: the worker counts devices itself, and only while HIP is not yet started."""
    monkeypatch.delenv(mp_util.NDEV_ENV, raising=False)
    monkeypatch.delenv("GPU_MAX_HW_QUEUES", raising=False)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    monkeypatch.setattr(torch.cuda, "set_device", lambda d: None)
    monkeypatch.setattr(torch.cuda, "is_initialized", lambda: False)
    assert mp_util.place_rank(1, 4) == (0, True) and os.environ["GPU_MAX_HW_QUEUES"] == "1"
    monkeypatch.setattr(torch.cuda, "is_initialized", lambda: True)
    with pytest.raises(AssertionError, match="initialisation"):
        mp_util.place_rank(1, 4)


def test_parent_exports_the_count(monkeypatch):
    monkeypatch.delenv(mp_util.NDEV_ENV, raising=False)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    assert mp_util.export_device_count() == 8 and os.environ[mp_util.NDEV_ENV] == "8"
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    assert mp_util.export_device_count() == 8  # idempotent: the first count stands


def _dies(code):
    os._exit(code)


def test_collect_fails_fast_on_a_dead_rank():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dies, args=(3,))]
    procs[0].start()
    with pytest.raises(pytest.fail.Exception, match="died without a result"):
        mp_util.collect(procs, q, 1, timeout=60)
