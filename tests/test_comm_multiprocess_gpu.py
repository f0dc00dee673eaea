"""Two (and 4, 8) processes, one rank each, all on cuda:0, through the NCCL ABI (ncclGetUniqueId ->
ncclCommInitRank -> ncclAllReduce): exercises the TCP bootstrap, hipIpc handle exchange of
scratch / semaphores / output buffers between processes, and every algorithm, checked bit-exactly
against the CPU oracle (same LCG inputs as test/torch/correctness_test.py:44-56)."""
import multiprocessing as mp
import os
import traceback

import numpy as np
import mp_util
import pytest

pytestmark = pytest.mark.gpu

CASES = [  # (algo, dtype code, count)
    ("allpair", 0, 4096), ("packet", 0, 1 << 18), ("fullmesh", 0, 1 << 20), ("rsag", 2, 100000),
    ("packet", 1, 30000), ("auto", 0, 48 << 19), ("auto", 2, 1000), ("fullmesh", 1, 12345),
    ("rsag_zc", 0, 1 << 20), ("rsag_zc", 2, 12345), ("rsag_pipeline", 2, 100000), ("rsag_pipeline", 2, 3 << 20),
    # 2 ranks: the selector's one-hop LL8 at the top of its range, default shape
    ("auto", 0, 1 << 19), ("auto", 0, (1 << 18) + 3),
]


def _worker(rank, n, uid, q, cases=None, rsag=True):
    try:
        os.environ.setdefault("MSCCLPP_AMD_SPIN_TIMEOUT_MS", "5000")
        import torch

        import mp_util
        import mscclpp_amd as m
        import oracle_lib as O

        mp_util.place_rank(rank, n)
        comm = m.Communicator(rank, n, uid)
        tdt = {0: torch.float16, 1: torch.bfloat16, 2: torch.float32}
        results = []
        for algo, dt, count in (cases or CASES):
            ins = [O.lcg(dt, count, r, 3) for r in range(n)]
            x = torch.from_numpy(ins[rank].view(np.int16 if dt < 2 else np.int32).copy()).view(tdt[dt]).cuda()
            out = torch.zeros_like(x)
            for _ in range(3):  # repeated calls: flag / semaphore lifecycle, registration cache
                comm.all_reduce(x, out, algo=None if algo == "auto" else algo)
            torch.cuda.synchronize()
            errc = comm.device_error()
            nbytes = count * (2 if dt < 2 else 4)
            sel = algo
            if algo == "auto":
                sel = {1: "packet", 2: "allpair", 3: "fullmesh"}[m.lib().mscclppAmdSelectAlgo(n, nbytes, dt)]
            if sel == "packet":
                exp, _ = O.allreduce_packet(dt, O.SUM, ins, count, 1, 1 << 22)
                e = exp[rank].view(np.uint8)[:nbytes]
            elif sel == "allpair":
                exp, _ = O.allreduce_allpairs(dt, O.SUM, ins, count, 1, 1 << 22)
                e = exp[rank].view(np.uint8)[:nbytes]
            else:
                sl = ((nbytes + n - 1) // n + 15) // 16 * 16
                nw = (nbytes + 3) // 4
                pad = []
                for a in ins:
                    w = np.zeros(nw, np.uint32)
                    w.view(np.uint8)[:nbytes] = a.view(np.uint8)
                    pad.append(w)
                e = O.allreduce_sliced(dt, O.SUM, pad, nw, sl // 4, 1 if sel in ("rsag", "rsag_zc") else 0)[rank].view(np.uint8)[:nbytes]
            got = out.cpu().contiguous().view(torch.uint8).numpy()
            results.append((algo, dt, count, errc, int(np.count_nonzero(got != e))))
        # ncclReduceScatter + ncclAllGather reconstruct the AllReduce (fp32, block 8192)
        block = 8192 if rsag else 0
        ins = [O.lcg(2, block * n, r, 9) for r in range(n)]
        x = torch.from_numpy(ins[rank].view(np.int32).copy()).view(torch.float32).cuda()
        rs = torch.zeros(block, dtype=torch.float32, device="cuda")
        ag = torch.zeros(block * n, dtype=torch.float32, device="cuda")
        if rsag:
            for _ in range(2):
                comm.reduce_scatter(x, rs)
                comm.all_gather(rs, ag)
            torch.cuda.synchronize()
            nw = block * n
            e = O.allreduce_sliced(2, O.SUM, [a.view(np.uint32) for a in ins], nw, block, 0)[0]
            got = ag.cpu().numpy().view(np.uint32)
            results.append(("rs+ag", 2, nw, comm.device_error(), int(np.count_nonzero(got != e))))
        comm.barrier()
        comm.destroy()
        q.put((rank, results, None))
    except Exception:
        q.put((rank, None, traceback.format_exc()))


def _run(n, cases=None, rsag=True, timeout=240):
    import mscclpp_amd as m

    uid = m.Communicator.unique_id()  # root thread lives in this (parent) process
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, n, uid, q, cases, rsag)) for r in range(n)]
    for p in procs:
        p.start()
    got = mp_util.collect(procs, q, n, timeout)
    for rank in range(n):
        for algo, dt, count, errc, bad in got[rank]:
            assert errc == 0, (rank, algo, dt, count, errc)
            assert bad == 0, (rank, algo, dt, count, bad)


def test_two_process_ncclallreduce(built):
    _run(2)


# 4 and 8 processes sharing one device: the rank counts the 8-GPU node runs (bootstrap with 8
# peers, 7 IPC mappings per buffer, the n = 4 / 8 slice geometries), at sizes whose launches from
# every rank fit on the device at once (the spinning kernels of all ranks must be co-resident).
MANY_CASES = [("allpair", 0, 4096), ("packet", 0, 1 << 17), ("packet", 1, 30001), ("fullmesh", 0, 1 << 19),
              ("rsag", 2, 100000), ("rsag_zc", 0, 1 << 19), ("auto", 2, 1000), ("auto", 0, 1 << 16)]


@pytest.mark.parametrize("n", [4, 8])
def test_many_process_ncclallreduce(built, n):
    _run(n, MANY_CASES, rsag=True, timeout=300)


def test_host_proxy_paths(built):
    """Config 1 (host-offload AllGather through the FIFO + proxy thread) and the PortChannel
    put / putWithSignal / putWithSignalAndFlush surface, 2 processes on cuda:0."""
    import sys as _s

    _s.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import host_proxy_baseline as H

    res = H.run(2, 4096, timeout=200)
    assert res["correct"], res
    assert res["us_per_kernel_graph"] > 0
    for mode, r in res["portchannel_alltoall_1MiB"].items():
        assert r["correct"], (mode, r)


def _ring_worker(rank, n, uid, q, nelems, nblocks):
    try:
        os.environ.setdefault("MSCCLPP_AMD_SPIN_TIMEOUT_MS", "20000")
        import torch

        import mscclpp_amd as m

        import mp_util

        mp_util.place_rank(rank, n)
        comm = m.Communicator(rank, n, uid)
        us, ok, _ = comm.proxy_ring_all_reduce(nelems, iters=1, graph_launches=1, nblocks=nblocks)
        errc = comm.device_error()
        comm.destroy()
        q.put((rank, (ok, errc), None))
    except Exception:
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.parametrize("nblocks", [2, 24])
def test_proxy_ring_reduced_halves_are_complete_before_put(built, nblocks):
    """mscclpp-test allreduce1 with 128 MiB halves and few workgroups: the sum of a half takes far
    longer than the proxy needs to start copying it, so a put triggered before every workgroup has
    finished its share of the sum (the reference's ordering, allreduce_test.cu:765-811) sends a
    partly reduced half.  The grid barrier before each such put must make the result exact."""
    import mscclpp_amd as m

    n = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    uid = m.Communicator.unique_id()
    procs = [ctx.Process(target=_ring_worker, args=(r, n, uid, q, 1 << 27, nblocks)) for r in range(n)]
    for p in procs:
        p.start()
    got = mp_util.collect(procs, q, n, 200)
    for rank in range(n):
        assert got[rank] == (True, 0), (rank, got[rank])


def _bcast_split_worker(rank, n, uid, q):
    try:
        os.environ.setdefault("MSCCLPP_AMD_SPIN_TIMEOUT_MS", "5000")
        import torch

        import mscclpp_amd as m

        import mp_util

        mp_util.place_rank(rank, n)
        comm = m.Communicator(rank, n, uid)
        out = []
        # ncclBroadcast out of place from the last rank, then ncclBcast in place from rank 0
        x = torch.arange(12345, dtype=torch.float32, device="cuda") * (rank + 1)
        y = torch.zeros_like(x)
        comm.broadcast(x, y, root=n - 1)
        torch.cuda.synchronize()
        out.append(bool(torch.equal(y, torch.arange(12345, dtype=torch.float32, device="cuda") * n)))
        z = torch.full((1 << 20,), float(rank), dtype=torch.float16, device="cuda")
        comm.broadcast(z, root=0)
        torch.cuda.synchronize()
        out.append(bool(torch.all(z == 0)))
        # ncclCommSplit: everyone in one color (same group, reversed order by key), then singletons
        sub = comm.split(0, n - 1 - rank)
        out.append(sub.rank == n - 1 - rank and sub.nranks == n)
        a = torch.full((4096,), float(sub.rank + 1), dtype=torch.float16, device="cuda")
        sub.all_reduce(a)
        torch.cuda.synchronize()
        out.append(bool(torch.all(a == n * (n + 1) / 2)))
        solo = comm.split(rank, 0)
        out.append(solo.nranks == 1 and solo.rank == 0)
        none = comm.split(-1 if rank == 0 else 5, 0)  # NCCL_SPLIT_NOCOLOR -> no communicator
        out.append((none is None) if rank == 0 else (none is not None and none.nranks == n - 1))
        for c in (sub, solo, none):
            if c is not None:
                c.destroy()
        out.append(comm.device_error())
        comm.destroy()
        q.put((rank, out, None))
    except Exception:
        q.put((rank, None, traceback.format_exc()))


def test_broadcast_and_split_two_processes(built):
    import mscclpp_amd as m

    n = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    uid = m.Communicator.unique_id()
    procs = [ctx.Process(target=_bcast_split_worker, args=(r, n, uid, q)) for r in range(n)]
    for p in procs:
        p.start()
    got = mp_util.collect(procs, q, n, 200)
    for rank in range(n):
        assert got[rank] == [True, True, True, True, True, True, 0], (rank, got[rank])


def _stream_order_worker(rank, n, uid, q):
    try:
        os.environ.setdefault("MSCCLPP_AMD_SPIN_TIMEOUT_MS", "10000")
        import torch

        import mscclpp_amd as m

        import mp_util

        mp_util.place_rank(rank, n)
        comm = m.Communicator(rank, n, uid)
        res = []
        blk = 1 << 18
        inp = torch.full((blk,), float(rank + 1), device="cuda")
        out = torch.empty(n * blk, device="cuda")
        exp = torch.cat([torch.full((blk,), float(r + 1), device="cuda") for r in range(n)])
        ar_in = torch.full((1 << 20,), float(rank + 1), dtype=torch.float16, device="cuda")
        ar_out = torch.empty_like(ar_in)
        for _ in range(3):
            # the receive buffers are still being written by this rank's own stream (a slow producer)
            # when the collective is enqueued behind it: peers must not write into them earlier
            torch.cuda._sleep(20_000_000)
            out.fill_(-1.0)
            comm.all_gather(inp, out)
            torch.cuda._sleep(20_000_000)
            ar_out.fill_(-1.0)
            comm.all_reduce(ar_in, ar_out, algo="rsag_zc")
            torch.cuda._sleep(20_000_000)
            ar_out.fill_(-1.0)
            comm.all_reduce(ar_in, ar_out, algo="fullmesh")
            torch.cuda.synchronize()
            res.append(bool(torch.equal(out, exp)) and bool(torch.all(ar_out == n * (n + 1) / 2)))
        res.append(comm.device_error())
        comm.destroy()
        q.put((rank, res, None))
    except Exception:
        q.put((rank, None, traceback.format_exc()))


def test_collectives_wait_for_the_peers_stream(built):
    """Remote writes into a peer's receive buffer start only after the peer's earlier stream work
    (which may still write that memory) is done: AllGather's entry handshake, and the handshakes that
    precede the output writes of the zero-copy and fullmesh AllReduce."""
    import mscclpp_amd as m

    n = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    uid = m.Communicator.unique_id()
    procs = [ctx.Process(target=_stream_order_worker, args=(r, n, uid, q)) for r in range(n)]
    for p in procs:
        p.start()
    got = mp_util.collect(procs, q, n, 200)
    for rank in range(n):
        assert got[rank] == [True, True, True, 0], (rank, got[rank])


def _pipeline_then_worker(rank, n, uid, q):
    try:
        os.environ.setdefault("MSCCLPP_AMD_SPIN_TIMEOUT_MS", "10000")
        import torch

        import mscclpp_amd as m

        import mp_util

        mp_util.place_rank(rank, n)
        comm = m.Communicator(rank, n, uid)
        res = []
        cnt = 3 << 20  # 12 MiB of int32: several pipeline iterations at every shape below
        base = torch.arange(cnt, dtype=torch.int32, device="cuda") % 1000003
        x = base + rank
        exp = base * n + n * (n - 1) // 2
        y = torch.empty_like(x)
        blk = 1 << 18
        rs_in = (torch.arange(n * blk, dtype=torch.int32, device="cuda") % 999) * (rank + 1)
        rs_out = torch.empty(blk, dtype=torch.int32, device="cuda")
        rs_exp = (torch.arange(n * blk, dtype=torch.int32, device="cuda") % 999)[rank * blk:(rank + 1) * blk] * (n * (n + 1) // 2)
        for it in range(6):
            nb, nt = ((32, 256), (64, 512), (2, 64))[it % 3]  # the geometry changes between calls
            y.fill_(-1)
            comm.all_reduce(x, y, algo="rsag_pipeline", nblocks=nb, nthreads=nt)
            # issued at once behind it on the same communicator: puts into the peers' bulk scratch
            comm.reduce_scatter(rs_in, rs_out)
            ok_pipe = bool(torch.equal(y, exp))
            y.fill_(-1)
            comm.all_reduce(x, y, algo="fullmesh", nblocks=64 if it % 2 else 128)
            comm.all_reduce(x, y, algo="rsag_pipeline", nblocks=nb, nthreads=nt)
            torch.cuda.synchronize()
            res.append(ok_pipe and bool(torch.equal(rs_out, rs_exp)) and bool(torch.equal(y, exp)))
        res.append(comm.device_error())
        comm.destroy()
        q.put((rank, res, None))
    except Exception:
        q.put((rank, None, traceback.format_exc()))


def test_pipeline_then_scratch_collectives(built):
    """the pipelined RS+AG must not end while a peer still copies out of its
    scratch, since the next collective on the communicator (reduce-scatter / fullmesh, which put into
    the peers' scratch with no entry handshake, or a pipeline of another geometry) reuses it."""
    import mscclpp_amd as m

    n = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    uid = m.Communicator.unique_id()
    procs = [ctx.Process(target=_pipeline_then_worker, args=(r, n, uid, q)) for r in range(n)]
    for p in procs:
        p.start()
    got = mp_util.collect(procs, q, n, 200)
    for rank in range(n):
        assert got[rank] == [True] * 6 + [0], (rank, got[rank])


def _churn_worker(rank, n, uid, q):
    try:
        os.environ.setdefault("MSCCLPP_AMD_SPIN_TIMEOUT_MS", "10000")
        import torch

        import mscclpp_amd as m

        import mp_util

        mp_util.place_rank(rank, n)
        comm = m.Communicator(rank, n, uid)
        L = m.lib()
        import ctypes

        bad, peak = 0, 0
        for it in range(1000):
            # a fresh device allocation per iteration, freed right after: hipMalloc hands the same
            # address back again and again, each time a new allocation (new IPC handle)
            p = ctypes.c_void_p()
            m.check(L.mscclppAmdMalloc(ctypes.byref(p), 1 << 20), "malloc")
            t = m.device_view(p.value, 1 << 20).view(torch.float32)
            t.fill_(float(rank + it))
            comm.all_reduce(t, t, algo="fullmesh" if it % 2 else "rsag_zc")
            torch.cuda.synchronize()
            exp = float(sum(r + it for r in range(n)))
            bad += int((t != exp).sum().item())
            regs, maps, retired = comm.registration_stats()
            peak = max(peak, regs)
            del t
            m.check(L.mscclppAmdFree(p), "free")
        regs, maps, retired = comm.registration_stats()
        err = comm.device_error()
        comm.destroy()
        q.put((rank, (bad, peak, maps, err), None))
    except Exception:
        q.put((rank, None, traceback.format_exc()))


def test_registration_churn_stays_bounded_and_exact(built):
    """1000 freshly allocated buffers through the zero-copy and fullmesh
    AllReduce (which register the user's buffers) stay exact without any explicit deregistration,
    and the registration cache stays bounded (a buffer re-allocated at the same address is a new
    registration; at most 64 stay registered)."""
    import mscclpp_amd as m

    n = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    uid = m.Communicator.unique_id()
    procs = [ctx.Process(target=_churn_worker, args=(r, n, uid, q)) for r in range(n)]
    for p in procs:
        p.start()
    got = mp_util.collect(procs, q, n, 240)
    for rank in range(n):
        bad, peak, maps, err = got[rank]
        assert bad == 0 and err == 0, (rank, got[rank])
        assert peak <= 64, (rank, got[rank])
        assert maps <= 80, (rank, got[rank])


def _symmetric_worker(rank, n, uid, symmetric, q):
    try:
        os.environ.setdefault("MSCCLPP_AMD_SPIN_TIMEOUT_MS", "10000")
        if symmetric:
            os.environ["MSCCLPP_NCCL_SYMMETRIC_MEMORY"] = "1"
        else:
            os.environ.pop("MSCCLPP_NCCL_SYMMETRIC_MEMORY", None)
        os.environ.pop("MSCCLPP_AMD_NCCL_SYMMETRIC_MEMORY", None)
        import ctypes

        import torch

        import mscclpp_amd as m

        import mp_util

        mp_util.place_rank(rank, n)
        comm = m.Communicator(rank, n, uid)
        L = m.lib()
        nslots, slot = 16, 1 << 19  # 16 sub-buffers of 512 KiB in one 8 MiB allocation
        p = ctypes.c_void_p()
        m.check(L.mscclppAmdMalloc(ctypes.byref(p), nslots * slot), "malloc")
        whole = m.device_view(p.value, nslots * slot).view(torch.float32)
        whole.fill_(-1.0)
        per = slot // 4
        bad = 0
        for rnd in range(2):
            for k in range(nslots):
                t = whole[k * per:(k + 1) * per]
                t.fill_(float(rank * 100 + k + rnd))
                comm.all_reduce(t, t, algo="fullmesh" if (k + rnd) % 2 else "rsag_zc")
            torch.cuda.synchronize()
            for k in range(nslots):
                exp = float(sum(r * 100 + k + rnd for r in range(n)))
                bad += int((whole[k * per:(k + 1) * per] != exp).sum().item())
        allocs, offs, sym = comm.registration_exchanges()
        err = comm.device_error()
        del whole
        comm.destroy()
        m.check(L.mscclppAmdFree(p), "free")
        q.put((rank, (bad, allocs, offs, sym, err), None))
    except Exception:
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.parametrize("symmetric", [True, False])
def test_symmetric_memory_registration(built, symmetric):
    """MSCCLPP_NCCL_SYMMETRIC_MEMORY (env.hpp:101-107): buffers at the same offset of one allocation
    on every rank.  16 sub-buffers of one allocation through fullmesh and zero-copy AllReduce (both
    register the user's buffers): exact either way; the allocation is exchanged once, and new offsets
    cost one host all-gather each only without the symmetric declaration."""
    import mscclpp_amd as m

    n = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    uid = m.Communicator.unique_id()
    procs = [ctx.Process(target=_symmetric_worker, args=(r, n, uid, symmetric, q)) for r in range(n)]
    for p in procs:
        p.start()
    got = mp_util.collect(procs, q, n, 180)
    for rank in range(n):
        bad, allocs, offs, sym, err = got[rank]
        assert bad == 0 and err == 0, (rank, got[rank])
        assert sym == symmetric
        assert allocs == 1, (rank, got[rank])
        assert offs == (0 if symmetric else 16), (rank, got[rank])


def _reimport_worker(rank, n, uid, q):
    try:
        os.environ.setdefault("MSCCLPP_AMD_SPIN_TIMEOUT_MS", "10000")
        import ctypes

        import torch

        import mscclpp_amd as m

        import mp_util

        mp_util.place_rank(rank, n)
        comm = m.Communicator(rank, n, uid)
        L = m.lib()
        bad, addrs = 0, set()
        for it in range(40):
            p = ctypes.c_void_p()
            m.check(L.mscclppAmdMalloc(ctypes.byref(p), 1 << 20), "malloc")
            addrs.add(p.value)
            t = m.device_view(p.value, 1 << 20).view(torch.float32)
            t.fill_(float(rank + 3 * it))
            comm.all_reduce(t, t, algo=("fullmesh", "rsag_zc", "rsag")[it % 3])
            torch.cuda.synchronize()
            bad += int((t != float(sum(r + 3 * it for r in range(n)))).sum().item())
            # every rank closes its imports of the peers' buffers BEFORE the peers free them and
            # allocate the next one (very likely at the same address): the next import of that
            # address must map the new memory
            comm.deregister_all()
            del t
            m.check(L.mscclppAmdFree(p), "free")
        err = comm.device_error()
        comm.destroy()
        q.put((rank, (bad, len(addrs), err), None))
    except Exception:
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.parametrize("n", [2, 4])
def test_reimport_after_close_at_the_same_address(built, n):
    """A peer buffer imported, closed, freed and re-allocated at the same address is imported
    afresh (the failure the scratch growth showed: an import of the new handle that mapped the old
    memory).  40 rounds over fullmesh / zero-copy / rsag, exact."""
    import mscclpp_amd as m

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    uid = m.Communicator.unique_id()
    procs = [ctx.Process(target=_reimport_worker, args=(r, n, uid, q)) for r in range(n)]
    for p in procs:
        p.start()
    got = mp_util.collect(procs, q, n, 180)
    for rank in range(n):
        bad, naddr, err = got[rank]
        assert bad == 0 and err == 0, (rank, got[rank])
