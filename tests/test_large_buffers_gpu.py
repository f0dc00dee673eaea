"""Buffers beyond 4 GiB (an MI355X holds 288 GB of HBM).  The kernels address memory through buffer
descriptors, whose offsets are 32 bits; the reference's kernels use 64-bit pointer arithmetic and
take any size.  Here:

* the MemoryChannel primitives (put, get, putPackets / unpackPackets in LL16 and LL8) walk a range of
  any size, rebasing their descriptor every 2 GiB (device.hpp for_each_strided): a 4 GiB + 3 MiB
  range comes back equal to its source pattern, which differs between words 4 GiB apart;
* the bulk AllReduce kernels stay within 4 GiB per descriptor: fullmesh / rsag cap a pass so the
  reduce step's n scratch regions fit (here a 2-rank 9 GiB bucket with 9 GiB of scratch runs in
  three passes instead of wrapping at 4 GiB), zero-copy and the pipeline address per workgroup;
  every int32 element of the result is checked against the sum of the inputs.
* the 1-GPU LL16 self-reduce (config 2) runs a 4.5 GiB bucket exactly; ReduceScatter, AllGather
  (4.5 GiB blocks) and Broadcast (9 GiB) likewise;
* ncclAllReduce between two processes (IPC-mapped 9 GiB buffers; default selector and rsag_zc);
* the LL protocols refuse buckets whose packet regions would pass 4 GiB (tests/test_library.py).
"""
import ctypes
import multiprocessing as mp
import os
import traceback

import pytest
import torch

pytestmark = pytest.mark.gpu

GiB, MiB = 1 << 30, 1 << 20


def _need(nbytes):
    free, _ = torch.cuda.mem_get_info()
    if free < nbytes:
        pytest.skip(f"needs {nbytes / GiB:.0f} GiB of free device memory")


def test_channel_primitives_beyond_4GiB(built):
    import mscclpp_amd as m

    nbytes = 4 * GiB + 3 * MiB + 48
    _need(5 * nbytes + 2 * GiB)
    L = m.lib()
    L.mscclppAmdMemChannelBigTest.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    bad = (ctypes.c_ulonglong * 4)()
    err = ctypes.c_uint32(0)
    rc = L.mscclppAmdMemChannelBigTest(nbytes, 1024, bad, ctypes.byref(err))
    assert rc == 0
    assert err.value == 0
    assert list(bad) == [0, 0, 0, 0], "words off after put, get, LL16 and LL8 round trips: %s" % list(bad)


@pytest.fixture(scope="module")
def big_ranks(built):
    import mscclpp_amd as m

    n, count = 2, (9 * GiB) // 4 + 4096  # int32 elements per rank: 9 GiB + 16 KiB
    nbytes = count * 4
    _need(5 * n * nbytes + 4 * GiB)
    ranks = m.InProcessRanks(n, 1 * MiB, nbytes)  # bulk scratch = the bucket: without the cap, one 4.5 GiB pass
    dev = torch.device("cuda", 0)
    ins = []
    for r in range(n):
        t = torch.empty(count, dtype=torch.int32, device=dev)
        for c in t.split(1 << 28):
            c.random_(0, 1 << 20)
        ins.append(t)
    outs = [torch.empty_like(t) for t in ins]
    yield m, ranks, ins, outs
    del ins, outs
    torch.cuda.empty_cache()


@pytest.mark.parametrize("algo", ["fullmesh", "rsag", "rsag_zc", "rsag_pipeline"])
def test_bulk_allreduce_beyond_4GiB(big_ranks, algo):
    m, ranks, ins, outs = big_ranks
    for o in outs:
        o.fill_(-1)
    torch.cuda.synchronize()
    ranks.all_reduce(ins, outs, m.ALGO_NAMES[algo], budget_ticks=3_000_000_000)
    torch.cuda.synchronize()
    assert ranks.errors() == [0] * ranks.n
    for r, o in enumerate(outs):
        wrong = 0
        for a, b, c in zip(ins[0].split(1 << 28), ins[1].split(1 << 28), o.split(1 << 28)):
            wrong += int((c != a + b).sum())
        assert wrong == 0, f"{algo}: rank {r} has {wrong} wrong int32 elements of {o.numel()}"


def test_self_reduce_beyond_4GiB(built):
    """The 1-GPU LL16 hot path (BASELINE config 2) on a 4.5 GiB int32 bucket: out = x + unpack(pack(y))
    for every element (the kernel rebases its descriptors per 1 KiB chunk)."""
    import mscclpp_amd as m

    count = (9 * GiB // 2) // 4 + 1024
    nbytes = count * 4
    _need(6 * nbytes + 2 * GiB)
    dev = torch.device("cuda", 0)
    x, y = (torch.empty(count, dtype=torch.int32, device=dev) for _ in range(2))
    for t in (x, y):
        for c in t.split(1 << 28):
            c.random_(0, 1 << 20)
    out = torch.full_like(x, -1)
    pk = m.DeviceBuffer(2 * nbytes)
    flags = torch.ones(m.FLAG_SLOTS, dtype=torch.int32, device=dev)
    err = torch.zeros(16, dtype=torch.int32, device=dev)
    m.self_reduce_ll16(x, y, pk.ptr, out, flags, err, budget_ticks=3_000_000_000)
    torch.cuda.synchronize()
    assert int(err[0]) == 0
    wrong = sum(int((c != a + b).sum()) for a, b, c in zip(x.split(1 << 28), y.split(1 << 28), out.split(1 << 28)))
    assert wrong == 0, f"{wrong} wrong int32 elements of {count}"
    pk.free()


@pytest.mark.parametrize("algo,nbytes", [("packet", 2 * GiB - MiB), ("allpair", GiB - MiB)])
def test_ll_at_largest_accepted_bucket(built, algo, nbytes):
    """LL16 / LL8 at 2 ranks just under their 4 GiB descriptor bound (packet regions reaching ~4 GiB
    from their base): every element right; one step above, the call is refused (ncclInvalidUsage)."""
    import mscclpp_amd as m

    n, code = 2, m.ALGO_NAMES[algo]
    sb = m.scratch_required(code, n, nbytes, m.I32)
    assert sb > 0 and m.scratch_required(code, n, nbytes + 2 * MiB, m.I32) == 0
    _need(n * (sb + 3 * nbytes) + 2 * GiB)
    dev = torch.device("cuda", 0)
    ranks = m.InProcessRanks(n, sb)
    ins = []
    for r in range(n):
        t = torch.empty(nbytes // 4, dtype=torch.int32, device=dev)
        for c in t.split(1 << 28):
            c.random_(0, 1 << 20)
        ins.append(t)
    outs = [torch.full_like(t, -1) for t in ins]
    ranks.all_reduce(ins, outs, code, budget_ticks=3_000_000_000)
    torch.cuda.synchronize()
    assert ranks.errors() == [0] * n
    for r, o in enumerate(outs):
        wrong = sum(int((c != a + b).sum()) for a, b, c in zip(ins[0].split(1 << 28), ins[1].split(1 << 28), o.split(1 << 28)))
        assert wrong == 0, f"{algo}: rank {r} has {wrong} wrong elements"
    del outs
    big = [torch.empty(nbytes // 4 + (2 * MiB) // 4, dtype=torch.int32, device=dev) for _ in range(n)]
    with pytest.raises(m.MscclppError):
        ranks.all_reduce(big, big, code)


@pytest.mark.parametrize("algo", ["fullmesh", "rsag"])
def test_reduce_scatter_and_all_gather_beyond_4GiB(big_ranks, algo):
    """ncclReduceScatter / ncclAllGather through the bulk kernel (modes 1 and 2) with 4.5 GiB blocks:
    9 GiB gathered or reduced per rank, in capped passes, every element checked."""
    m, ranks, ins, outs = big_ranks
    n = ranks.n
    block = (ins[0].numel() // n) // 4 * 4  # int32 elements per rank block (16-byte multiple)
    chunk = 1 << 28
    # ReduceScatter: rank r gets sum over q of ins[q][r*block : (r+1)*block]
    rs_in = [t[: n * block] for t in ins]
    rs_out = [o[:block] for o in outs]
    for o in rs_out:
        o.fill_(-1)
    ranks.collective(1, rs_in, rs_out, algo=m.ALGO_NAMES[algo], budget_ticks=3_000_000_000)
    torch.cuda.synchronize()
    assert ranks.errors() == [0] * n
    for r in range(n):
        lo = r * block
        wrong = 0
        for s in range(0, block, chunk):
            e = min(block, s + chunk)
            wrong += int((rs_out[r][s:e] != ins[0][lo + s:lo + e] + ins[1][lo + s:lo + e]).sum())
        assert wrong == 0, f"ReduceScatter {algo}: rank {r} has {wrong} wrong elements"
    # AllGather: outs[r] = ins[0][:block] ++ ins[1][:block]
    ag_in = [t[:block] for t in ins]
    ag_out = [o[: n * block] for o in outs]
    for o in ag_out:
        o.fill_(-1)
    ranks.collective(2, ag_in, ag_out, algo=m.ALGO_NAMES[algo], budget_ticks=3_000_000_000)
    torch.cuda.synchronize()
    assert ranks.errors() == [0] * n
    for r in range(n):
        wrong = 0
        for q in range(n):
            for s in range(0, block, chunk):
                e = min(block, s + chunk)
                wrong += int((ag_out[r][q * block + s:q * block + e] != ins[q][s:e]).sum())
        assert wrong == 0, f"AllGather {algo}: rank {r} has {wrong} wrong elements"


def test_broadcast_beyond_4GiB(big_ranks):
    """ncclBroadcast's zero-copy pull of a 9 GiB buffer from root 1 (default shape: 128 workgroups)."""
    m, ranks, ins, outs = big_ranks
    for o in outs:
        o.fill_(-1)
    ranks.broadcast(ins, outs, 1, budget_ticks=3_000_000_000)
    torch.cuda.synchronize()
    assert ranks.errors() == [0] * ranks.n
    for r, o in enumerate(outs):
        wrong = sum(int((c != a).sum()) for a, c in zip(ins[1].split(1 << 28), o.split(1 << 28)))
        assert wrong == 0, f"rank {r} has {wrong} wrong elements"


def _pattern(rank, lo, hi, device):
    """int32 elements [lo, hi) of rank's input: distinct 4 GiB apart, small enough that sums stay exact."""
    i = torch.arange(lo, hi, dtype=torch.int64, device=device)
    return ((i * 2654435761 + (i >> 30) * 97 + rank * 12345) & 0xFFFFF).to(torch.int32)


def _nccl_worker(rank, n, uid, count, q):
    try:
        os.environ.setdefault("MSCCLPP_AMD_SPIN_TIMEOUT_MS", "20000")
        import mp_util

        mp_util.place_rank(rank, n)
        import mscclpp_amd as m

        dev = torch.device("cuda", torch.cuda.current_device())
        comm = m.Communicator(rank, n, uid)
        chunk = 1 << 28
        x = torch.empty(count, dtype=torch.int32, device=dev)
        for s in range(0, count, chunk):
            x[s:s + chunk] = _pattern(rank, s, min(count, s + chunk), dev)
        out = torch.empty_like(x)
        res = []
        for algo in (None, "rsag_zc"):  # the selector's choice at 9 GiB (fullmesh, many 128 MiB-scratch passes), zero-copy
            out.fill_(-1)
            comm.all_reduce(x, out, algo=algo)
            torch.cuda.synchronize()
            wrong = 0
            for s in range(0, count, chunk):
                e = min(count, s + chunk)
                want = sum(_pattern(r, s, e, dev) for r in range(n))
                wrong += int((out[s:e] != want).sum())
            res.append((algo or "auto", comm.device_error(), wrong))
        comm.barrier()
        comm.destroy()
        q.put((rank, res, None))
    except Exception:
        q.put((rank, None, traceback.format_exc()))


def test_nccl_allreduce_two_processes_beyond_4GiB(built):
    """The drop-in path end to end: ncclAllReduce between two processes (IPC-mapped 9 GiB outputs
    and inputs) -- the default selector (fullmesh through the communicator's 128 MiB scratch) and
    zero-copy rsag -- every element equal to the sum of both ranks' inputs."""
    import mp_util
    import mscclpp_amd as m

    n, count = 2, (9 * GiB) // 4 + 4096
    _need(n * (2 * count * 4 + 3 * GiB))
    uid = m.Communicator.unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_nccl_worker, args=(r, n, uid, count, q)) for r in range(n)]
    for p in procs:
        p.start()
    got = mp_util.collect(procs, q, n, 240)
    for rank in range(n):
        for algo, errc, wrong in got[rank]:
            assert errc == 0 and wrong == 0, (rank, algo, errc, wrong)
