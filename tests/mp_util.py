"""Rank placement for the multi-process GPU tests: rank r on device r % device_count, so the same
suite puts one rank on each GPU of a node (every byte between ranks then crosses xGMI, as in the
reference's mp_unit tests, test/mp_unit/mp_unit_tests.cc:109-121) and shares device 0 on a one-GPU
box (a rehearsal of the same protocol through local HBM).  torch.cuda.device_count() does not
initialise HIP, so a worker may call this before anything else touches the GPU."""
import os


def place_rank(rank, n):
    """Set this rank's device; returns (device index, shared).  With more than two ranks on one
    device, every rank process gets one hardware queue (set before HIP starts) so every rank's queue
    stays mapped while their spinning kernels wait for each other."""
    import torch

    ndev = torch.cuda.device_count()
    shared = ndev < n
    if shared and n > 2:
        os.environ["GPU_MAX_HW_QUEUES"] = "1"
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
