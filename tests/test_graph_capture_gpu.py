"""AllReduce captured in a HIP graph (torch.cuda.CUDAGraph) and replayed with new data, two processes
through the NCCL ABI: the way frameworks run collectives inside captured steps, and the way the
reference's harness times them (test/mscclpp-test/common.cc:202-227); ncclReduceScatter and
ncclAllGather are captured together as well.  Every replay must read the
inputs as they are at replay time and produce the oracle's bits: the LL flags and the bulk
semaphore counters live in device memory and advance inside the kernels, so nothing captured goes
stale between replays.  Buffers are registered by one eager call before the capture (a new buffer
costs a host exchange, which has no place inside a capture)."""
import multiprocessing as mp
import ctypes
import traceback

import numpy as np
import mp_util
import pytest

pytestmark = pytest.mark.gpu

CASES = [("allpair", 0, 4096), ("packet", 0, 1 << 17), ("fullmesh", 0, 1 << 20), ("rsag", 2, 100000),
         ("rsag_zc", 0, 1 << 20), ("rsag_pipeline", 2, 1 << 18)]
REPLAYS = 3


def _expected(O, algo, dt, count, ins, rank, n):
    nbytes = count * (2 if dt < 2 else 4)
    if algo == "packet":
        exp, _ = O.allreduce_packet(dt, O.SUM, ins, count, 1, 1 << 22)
        return exp[rank].view(np.uint8)[:nbytes]
    if algo == "allpair":
        exp, _ = O.allreduce_allpairs(dt, O.SUM, ins, count, 1, 1 << 22)
        return exp[rank].view(np.uint8)[:nbytes]
    nw = (nbytes + 3) // 4
    pad = []
    for a in ins:
        w = np.zeros(nw, np.uint32)
        w.view(np.uint8)[:nbytes] = a.view(np.uint8)
        pad.append(w)
    if algo == "rsag_pipeline":
        return None  # interleaved ownership: checked against fp32 sums with the tolerance below
    sl = ((nbytes + n - 1) // n + 15) // 16 * 16
    order = 1 if algo in ("rsag", "rsag_zc") else 0
    return O.allreduce_sliced(dt, O.SUM, pad, nw, sl // 4, order)[rank].view(np.uint8)[:nbytes]


def _worker(rank, n, uid, q):
    try:
        import os

        os.environ.setdefault("MSCCLPP_AMD_SPIN_TIMEOUT_MS", "5000")
        import torch

        import mscclpp_amd as m
        import oracle_lib as O

        import mp_util

        mp_util.place_rank(rank, n)
        comm = m.Communicator(rank, n, uid)
        tdt = {0: torch.float16, 2: torch.float32}
        out = []
        for algo, dt, count in CASES:
            x = torch.zeros(count, dtype=tdt[dt], device="cuda")
            y = torch.zeros_like(x)
            comm.all_reduce(x, y, algo=algo)  # registers x and y (host exchange) outside the capture
            torch.cuda.synchronize()
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=side):
                comm.all_reduce(x, y, algo=algo)
            torch.cuda.synchronize()
            bad = []
            for k in range(REPLAYS):
                ins = [O.lcg(dt, count, r, 20 + k) for r in range(n)]
                x.copy_(torch.from_numpy(ins[rank].view(np.int16 if dt < 2 else np.int32).copy()).view(tdt[dt]))
                y.fill_(-1)
                torch.cuda.synchronize()
                g.replay()
                torch.cuda.synchronize()
                got = y.cpu().contiguous().view(torch.uint8).numpy()
                e = _expected(O, algo, dt, count, ins, rank, n)
                if e is None:
                    ref = sum(a.view(np.float32).astype(np.float64) for a in ins)
                    ok = np.allclose(got.view(np.float32), ref, rtol=1e-5, atol=1e-5)
                    bad.append(0 if ok else 1)
                else:
                    bad.append(int(np.count_nonzero(got != e)))
            out.append((algo, bad, comm.device_error()))
            del g
        # ncclReduceScatter then ncclAllGather (fp32, block 8192) captured together
        block = 8192
        x = torch.zeros(block * n, dtype=torch.float32, device="cuda")
        rs = torch.zeros(block, dtype=torch.float32, device="cuda")
        ag = torch.zeros(block * n, dtype=torch.float32, device="cuda")
        comm.reduce_scatter(x, rs)
        comm.all_gather(rs, ag)
        torch.cuda.synchronize()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            comm.reduce_scatter(x, rs)
            comm.all_gather(rs, ag)
        torch.cuda.synchronize()
        bad = []
        for k in range(REPLAYS):
            ins = [O.lcg(2, block * n, r, 60 + k) for r in range(n)]
            x.copy_(torch.from_numpy(ins[rank].view(np.int32).copy()).view(torch.float32))
            rs.fill_(-1)
            ag.fill_(-1)
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            e = O.allreduce_sliced(2, O.SUM, [a.view(np.uint32) for a in ins], block * n, block, 0)[0]
            got_ag = ag.cpu().numpy().view(np.uint32)
            got_rs = rs.cpu().numpy().view(np.uint32)
            bad.append(int(np.count_nonzero(got_ag != e)) + int(np.count_nonzero(got_rs != e[rank * block:(rank + 1) * block])))
        out.append(("reducescatter+allgather", bad, comm.device_error()))
        del g
        comm.barrier()
        comm.destroy()
        q.put((rank, out, None))
    except Exception:
        q.put((rank, None, traceback.format_exc()))


def test_captured_allreduce_replays_with_new_data(built):
    import mscclpp_amd as m

    n = 2
    uid = m.Communicator.unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, n, uid, q)) for r in range(n)]
    for p in procs:
        p.start()
    got = mp_util.collect(procs, q, n, 240)
    for rank in range(n):
        for algo, bad, errc in got[rank]:
            assert errc == 0, (rank, algo, errc)
            assert bad == [0] * REPLAYS, (rank, algo, bad)


def _churn_worker(rank, n, uid, q):
    try:
        import os

        os.environ.setdefault("MSCCLPP_AMD_SPIN_TIMEOUT_MS", "5000")
        os.environ["MSCCLPP_AMD_MAX_USER_REGS"] = "64"  # 70 allocations below must evict
        import torch

        import mscclpp_amd as m
        import oracle_lib as O

        import mp_util

        mp_util.place_rank(rank, n)
        comm = m.Communicator(rank, n, uid)
        count = 6 << 20  # 12 MiB: above the caching allocator's 10 MiB packing, so its own segment
        # a buffer registered for the caller (an algorithm plugin keeps these raw peer pointers)
        z = torch.zeros(count, dtype=torch.int16, device="cuda")
        pz = comm.register_buffer(z)
        x = torch.zeros(count, dtype=torch.float16, device="cuda")
        y = torch.zeros_like(x)
        comm.all_reduce(x, y, algo="rsag_zc")
        torch.cuda.synchronize()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            comm.all_reduce(x, y, algo="rsag_zc")  # pins x's and y's registrations
        torch.cuda.synchronize()
        pinned = comm.registration_stats()[0]
        # a captured broadcast from root 0, then an eager one from another root buffer: the eager
        # call replaces the root's mapping, which the graph still reads through on replay
        bsrc = torch.zeros(count, dtype=torch.int32, device="cuda")
        bsrc2 = torch.zeros_like(bsrc)
        brecv = torch.zeros_like(bsrc)
        comm.broadcast(bsrc, brecv, root=0)
        torch.cuda.synchronize()
        gb = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gb, stream=side):
            comm.broadcast(bsrc, brecv, root=0, stream=side)
        torch.cuda.synchronize()
        comm.broadcast(bsrc2, brecv, root=0)
        torch.cuda.synchronize()
        # more fresh allocations than the registration cache holds (64), each its own segment
        keep = []
        for i in range(70):
            a = torch.full((6 << 20,), float(i % 7), dtype=torch.float16, device="cuda")
            b = torch.empty_like(a)
            comm.all_reduce(a, b, algo="rsag_zc")
            keep.append((a, b))
        torch.cuda.synchronize()
        regs, live, retired = comm.registration_stats()
        res = {"regs": regs, "pinned": pinned}
        if pinned >= 1 and regs == 64 + pinned:  # every pinned registration survived: replaying is safe
            ins = [O.lcg(O.F16, count, r, 77) for r in range(n)]
            x.copy_(torch.from_numpy(ins[rank].view(np.int16).copy()).view(torch.float16))
            y.fill_(-1)
            torch.cuda.synchronize()
            comm.barrier()
            g.replay()
            torch.cuda.synchronize()
            e = _expected(O, "rsag_zc", 0, count, ins, rank, n)
            res["bad"] = int(np.count_nonzero(y.cpu().contiguous().view(torch.uint8).numpy() != e))
            res["err"] = comm.device_error()
        # the captured broadcast replays through the root's old mapping, on new data
        if rank == 0:
            bsrc.copy_(torch.arange(count, dtype=torch.int32, device="cuda"))
        brecv.fill_(-1)
        torch.cuda.synchronize()
        comm.barrier()
        gb.replay()
        torch.cuda.synchronize()
        comm.barrier()
        want = torch.arange(count, dtype=torch.int32, device="cuda")
        res["bcast_bad"] = int((brecv != want).sum().item())
        # the caller's registration is still mapped after the churn: write a pattern into the next
        # rank's z through the pointer registered before it (a plugin's use), check on the owner
        src = torch.full((count,), 100 + rank, dtype=torch.int16, device="cuda")
        L = m.lib()
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        m.check(L.mscclppAmdCopyJobsPolicy((vp * 1)(src.data_ptr()), (vp * 1)(pz[(rank + 1) % n]),
                                           (sz * 1)(2 * count), 1, 64, 0, 0, m.stream_ptr()), "copy jobs")
        torch.cuda.synchronize()
        comm.barrier()
        res["registered_bad"] = int((z != 100 + (rank - 1) % n).sum().item())
        res["err2"] = comm.device_error()
        del g, gb, keep
        comm.barrier()
        comm.destroy()
        q.put((rank, res, None))
    except Exception:
        q.put((rank, None, traceback.format_exc()))


def test_captured_buffers_survive_registration_churn(built):
    """A graph keeps the peer pointers of its buffers: their registrations must not be evicted by
    later eager calls on 140 other buffers (the cache is bounded at 64 here), or the replay would write through
    closed mappings.  The pin is checked through the registration count before anything replays."""
    import mscclpp_amd as m

    n = 2
    uid = m.Communicator.unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_churn_worker, args=(r, n, uid, q)) for r in range(n)]
    for p in procs:
        p.start()
    got = mp_util.collect(procs, q, n, 240)
    for rank in range(n):
        assert got[rank]["pinned"] >= 1 and got[rank]["regs"] == 64 + got[rank]["pinned"], got
        assert got[rank]["bad"] == 0 and got[rank]["err"] == 0, got
        assert got[rank]["bcast_bad"] == 0 and got[rank]["registered_bad"] == 0 and got[rank]["err2"] == 0, got
