"""CPU, world_size 2 and 4 with the gloo backend: the N>1 setup path of bench.py / Communicator --
rank 0 creates the unique id (ncclGetUniqueId), torch.distributed broadcasts it, every rank joins
the library's TCP bootstrap and runs all-gather / barrier rounds (what ncclCommInitRank does
before any device work), and the max-over-ranks timing reduction of bench.py."""
import ctypes
import os
import socket

import pytest
import torch.multiprocessing as tmp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import numpy as np
    import torch
    import torch.distributed as dist

    import mscclpp_amd as m

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    L = m.lib()
    L.mscclppAmdBootstrapCreate.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)]
    L.mscclppAmdBootstrapAllGather.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    L.mscclppAmdBootstrapBarrier.argtypes = [ctypes.c_void_p]
    L.mscclppAmdBootstrapDestroy.argtypes = [ctypes.c_void_p]
    obj = [m.Communicator.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    h = ctypes.c_void_p()
    assert L.mscclppAmdBootstrapCreate(rank, world, obj[0], ctypes.byref(h)) == 0
    ok = True
    for rnd in range(3):
        mine = np.full(16, rank * 100 + rnd, dtype=np.int64)
        allv = np.zeros(16 * world, dtype=np.int64)
        assert L.mscclppAmdBootstrapAllGather(h, mine.ctypes.data, allv.ctypes.data, mine.nbytes) == 0
        for r in range(world):
            ok &= bool(np.all(allv[16 * r:16 * (r + 1)] == r * 100 + rnd))
        assert L.mscclppAmdBootstrapBarrier(h) == 0
    # bench.py's max-over-ranks reduction of per-rank step times
    t = torch.tensor([0.001 * (rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ok &= abs(float(t[0]) - 0.001 * world) < 1e-12
    L.mscclppAmdBootstrapDestroy(h)
    dist.destroy_process_group()
    q.put((rank, ok))


@pytest.mark.parametrize("world", [2, 4])
def test_bootstrap_over_gloo(built, world):
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=30)
    assert all(res[r] for r in range(world)), res
