"""Rank placement for the multi-process GPU tests: rank r on device r % device_count, so the same
suite puts one rank on each GPU of a node (every byte between ranks then crosses xGMI, as in the
reference's mp_unit tests, test/mp_unit/mp_unit_tests.cc:109-121) and shares device 0 on a one-GPU
box (a rehearsal of the same protocol through local HBM).

The device count comes from the PARENT (tests/conftest.py exports MSCCLPP_AMD_TEST_NDEV before any
rank process is spawned), because a worker must decide GPU_MAX_HW_QUEUES before HIP starts: HIP
reads its GPU_* flags once, at runtime initialisation, and torch.cuda.device_count() may itself
start the runtime (hipGetDeviceCount) when amdsmi cannot answer, which would ignore the setting."""
import os

NDEV_ENV = "MSCCLPP_AMD_TEST_NDEV"


def export_device_count():
    """Parent side: record the device count for rank processes spawned later (idempotent)."""
    if NDEV_ENV not in os.environ:
        import torch

        os.environ[NDEV_ENV] = str(torch.cuda.device_count())
    return int(os.environ[NDEV_ENV])


def queues_for(n, ndev):
    """GPU_MAX_HW_QUEUES a rank process needs, or None: with more than two ranks on one device every
    rank gets one hardware queue, so every rank's queue stays mapped while their spinning kernels
    wait for each other."""
    return "1" if ndev < n and n > 2 else None


def place_rank(rank, n):
    """Set this rank's device; returns (device index, shared).  Sets GPU_MAX_HW_QUEUES (queues_for)
    before anything here touches HIP; fails loudly when the parent did not export the device count
    and the runtime has already been started in this process, since the setting would be ignored."""
    ndev_env = os.environ.get(NDEV_ENV)
    if ndev_env is not None:
        ndev = int(ndev_env)
        q = queues_for(n, ndev)
        if q is not None:
            os.environ["GPU_MAX_HW_QUEUES"] = q
        import torch
    else:
        import torch

        assert not torch.cuda.is_initialized(), "place_rank after CUDA/HIP initialisation: queue setting would be lost"
        ndev = torch.cuda.device_count()
        q = queues_for(n, ndev)
        if q is not None:
            os.environ["GPU_MAX_HW_QUEUES"] = q
    shared = ndev < n
    dev = rank % max(1, ndev)
    torch.cuda.set_device(dev)
    return dev, shared


def collect(procs, q, n, timeout):
    """The (rank -> result) of n rank processes that put (rank, result, error) on q.  Fails at once
    when a rank reported an error or died without reporting (a crash, a segfault), instead of
    waiting out the timeout; kills what is left at the end."""
    import queue
    import time

    import pytest

    got, deadline = {}, time.time() + timeout
    try:
        while len(got) < n:
            try:
                rank, res, err = q.get(timeout=2)
            except queue.Empty:
                dead = [(i, p.exitcode) for i, p in enumerate(procs) if p.exitcode not in (None, 0) and i not in got]
                if dead:
                    pytest.fail(f"rank process(es) died without a result: {dead}")
                if time.time() > deadline:
                    pytest.fail(f"timed out after {timeout} s; results from ranks {sorted(got)}")
                continue
            assert err is None, f"rank {rank}: {err}"
            got[rank] = res
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return got
