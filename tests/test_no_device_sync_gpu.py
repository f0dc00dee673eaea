"""No device-wide synchronize on the call path.

Two rank processes cycle 70 distinct output allocations -- more than a registration cache bounded at 64 (MSCCLPP_AMD_MAX_USER_REGS=64), so
the least recently used registrations are retired while the calls go on -- through ncclAllReduce
while a long kernel (torch.cuda._sleep, ~3 s) runs on another stream of the same device.  A retired
mapping now closes when the events recorded after its last launches have completed
(comm_internal.hpp flushRetired), and a freed pooled block waits in the pool's pending list instead
of synchronizing (uncached_pool.cpp): so the 70 calls and 8 frees of pooled blocks return while the
other stream is still busy, and every one of the 70 results is bit-exact against the CPU oracle.
Then the first 8 (evicted) outputs are used again while their old mappings are still queued for
closing or being closed, and their new results are bit-exact too.
The reference's context cache never synchronizes either (src/core/algorithm.cc:52-60)."""
import multiprocessing as mp
import os
import time
import traceback

import numpy as np
import pytest

import mp_util

pytestmark = pytest.mark.gpu

NBUF = 70
NREUSE = 8  # evicted outputs used again while their mappings are being closed
COUNT = (1 << 20) + 512  # fp16: 2 MiB + 1 KiB, above the LL range at 2 ranks: a registering bulk kernel


def _worker(rank, n, uid, cap, q):
    try:
        os.environ.setdefault("MSCCLPP_AMD_SPIN_TIMEOUT_MS", "20000")
        os.environ["MSCCLPP_AMD_MAX_USER_REGS"] = str(cap)
        import torch

        import mp_util
        import mscclpp_amd as m
        import oracle_lib as O

        mp_util.place_rank(rank, n)
        comm = m.Communicator(rank, n, uid)
        nbytes = COUNT * 2
        sel = m.lib().mscclppAmdSelectAlgo(n, nbytes, 0)
        ins = [O.lcg(O.F16, COUNT, r, 11) for r in range(n)]
        x = torch.from_numpy(ins[rank].view(np.int16).copy()).view(torch.float16).cuda()
        # one hipMalloc per output (torch's allocator would carve several tensors from one segment,
        # i.e. one registration): 70 distinct allocations
        bufs = [m.DeviceBuffer(nbytes, uncached=False) for _ in range(NBUF)]
        outs = [m.device_view(b.ptr, nbytes).view(torch.float16) for b in bufs]
        for o in outs:
            o.fill_(float("nan"))
        pooled = [m.DeviceBuffer(1 << 20) for _ in range(8)]
        side = torch.cuda.Stream()
        # calibrate the spin kernel: cycles per ms on this device
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(side):
            a.record()
            torch.cuda._sleep(50_000_000)
            b.record()
        torch.cuda.synchronize()
        cycles_per_ms = 50_000_000 / max(a.elapsed_time(b), 1e-3)
        sleep_ms = 3000.0
        comm.barrier()
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(side):
            s0.record()
            torch.cuda._sleep(int(cycles_per_ms * sleep_ms))
            s1.record()
        fds0 = len(os.listdir("/proc/self/fd"))
        t0 = time.perf_counter()
        per_call = []
        for o in outs:
            tc = time.perf_counter()
            comm.all_reduce(x, o)  # ncclAllReduce: no algorithm, the library's selector
            per_call.append(time.perf_counter() - tc)
        t_calls = time.perf_counter() - t0
        fds1 = len(os.listdir("/proc/self/fd"))  # diagnosis: file descriptors the 70 registrations hold
        busy_after_calls = not s1.query()  # the event after the sleep has not completed
        t1 = time.perf_counter()
        for p in pooled:
            p.free()
        t_frees = time.perf_counter() - t1
        busy_after_frees = not s1.query()
        regs, _, awaiting = comm.registration_stats()
        # re-use the first evicted outputs while the sleep still runs: their old mappings are queued
        # for closing or being closed (the closer thread waits in hipIpcCloseMemHandle for the device
        # to go idle), so re-registering them revives a queued mapping or waits for the close in
        # flight (core.cpp openIpcHandle) -- never opens a handle that is half torn down
        ins2 = [O.lcg(O.F16, COUNT, r, 12) for r in range(n)]
        x2 = torch.from_numpy(ins2[rank].view(np.int16).copy()).view(torch.float16).cuda()
        ex_before = comm.registration_exchanges()[0]  # allocations registered so far (host exchanges)
        t2 = time.perf_counter()
        for o in outs[:NREUSE]:
            comm.all_reduce(x2, o)
        t_reuse = time.perf_counter() - t2  # diagnosis: includes any wait for a close in flight
        exchanges = (ex_before, comm.registration_exchanges()[0] - ex_before)
        torch.cuda.synchronize()
        slept_ms = s0.elapsed_time(s1)
        _, _, awaiting_after = comm.registration_stats()
        errc = comm.device_error()
        nw = (nbytes + 3) // 4
        sl = ((nbytes + n - 1) // n + 15) // 16 * 16
        pad = []
        for arr in ins:
            w = np.zeros(nw, np.uint32)
            w.view(np.uint8)[:nbytes] = arr.view(np.uint8)
            pad.append(w)
        # two ranks: x0 + x1 == x1 + x0, so fullmesh and the ring orders give the same words
        exp = O.allreduce_sliced(O.F16, O.SUM, pad, nw, sl // 4, 0)[rank].view(np.uint8)[:nbytes]
        pad2 = []
        for arr in ins2:
            w = np.zeros(nw, np.uint32)
            w.view(np.uint8)[:nbytes] = arr.view(np.uint8)
            pad2.append(w)
        exp2 = O.allreduce_sliced(O.F16, O.SUM, pad2, nw, sl // 4, 0)[rank].view(np.uint8)[:nbytes]
        bad = [i for i, o in enumerate(outs)
               if not np.array_equal(o.cpu().view(torch.uint8).numpy(), exp2 if i < NREUSE else exp)]
        comm.barrier()
        comm.destroy()
        for b_ in bufs:
            b_.free()
        q.put((rank, {"sel": sel, "cycles_per_ms": cycles_per_ms, "t_calls": t_calls, "t_frees": t_frees,
                      "busy_after_calls": busy_after_calls, "slept_ms": slept_ms,
                      "slowest_call": (max(per_call), per_call.index(max(per_call))),
                      "calls_over_10ms": [i for i, t in enumerate(per_call) if t > 0.01], "busy_after_frees": busy_after_frees, "regs": regs,
                      "awaiting": awaiting, "fds": (fds0, fds1), "t_reuse": t_reuse, "exchanges": exchanges, "awaiting_after": awaiting_after, "err": errc, "bad": bad}, None))
    except Exception:
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.parametrize("cap", [64, 128])
def test_calls_and_frees_do_not_wait_for_other_streams(built, cap):
    """cap 64 (the default): the calls evict registrations; MSCCLPP_AMD_MAX_USER_REGS=128: they do not,
    and the reuse pass registers nothing."""
    import mscclpp_amd as m

    n = 2
    uid = m.Communicator.unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, n, uid, cap, q)) for r in range(n)]
    for p in procs:
        p.start()
    got = mp_util.collect(procs, q, n, 240)
    print({rank: r for rank, r in got.items()})
    for rank, r in got.items():
        assert r["sel"] == 3, r  # fullmesh: a bulk algorithm that registers its output, not the LL paths
        assert r["err"] == 0 and r["bad"] == [], (rank, r)
        # fullmesh registers its output only: one exchange per new output allocation
        if cap == 64:  # the calls evicted registrations (70 > 64) without joining the sleeping stream
            assert r["regs"] <= 64 + 1 and r["exchanges"] == (NBUF, NREUSE), (rank, r)
        else:  # all 70 stay registered: the reuse pass is a cache hit on every rank
            assert r["regs"] == NBUF and r["exchanges"] == (NBUF, 0), (rank, r)
        assert r["busy_after_calls"] and r["busy_after_frees"], f"rank {rank}: {r}"
        # and no call waited for it: the 70 calls took a fraction of the sleep
        assert r["t_calls"] < 0.25 * r["slept_ms"] * 1e-3 and r["t_frees"] < 0.5, f"rank {rank}: {r}"
        assert r["awaiting_after"] == 0, (rank, r)  # everything retired closed once the device drained
