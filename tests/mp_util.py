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
