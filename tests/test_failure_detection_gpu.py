"""Failure detection: a peer that never joins a collective must end as an error the
caller can read, never as a hang.  Every wait in the kernels is bounded by a time budget
(s_memrealtime ticks, MSCCLPP_AMD_SPIN_TIMEOUT_MS on a communicator); on expiry the first waiter
records its reason in the rank's error word (kErrPacketTimeout = 1 for an LL packet,
kErrSemaphoreTimeout = 2 with channel / peer / rank / token detail for a handshake) and the kernel
runs to its end.  The reference's waits spin without a bound (semaphore_device.hpp:72-75,
packet_device.hpp:88-92 in release builds); NCCL's contract for this case is
ncclCommGetAsyncError -> ncclRemoteError, which is what the communicator reports here.

In-process cases launch rank 0 of a 2-rank AllReduce alone (one view): its peer's scratch, tokens
and buffers exist but no kernel of the peer ever runs.  The two-process case runs the NCCL ABI with
rank 1 never calling the collective."""
import multiprocessing as mp
import time
import traceback

import mp_util
import pytest
import torch

pytestmark = pytest.mark.gpu

ERR_PACKET_TIMEOUT, ERR_SEMAPHORE_TIMEOUT = 1, 2
BUDGET_TICKS = 20_000_000  # 0.2 s at the 100 MHz s_memrealtime clock


@pytest.mark.parametrize("algo_name,count,code", [
    ("allpair", 512, ERR_PACKET_TIMEOUT),
    ("packet", 1 << 16, ERR_PACKET_TIMEOUT),
    ("fullmesh", 1 << 16, ERR_SEMAPHORE_TIMEOUT),
    ("rsag_zc", 1 << 16, ERR_SEMAPHORE_TIMEOUT),
])
def test_absent_peer_ends_in_error_word(built, algo_name, count, code):
    import mscclpp_amd as m

    torch.cuda.set_device(0)
    algo = m.ALGO_NAMES[algo_name]
    n = 2
    nbytes = count * 2
    sb = max(m.scratch_required(m.ALGO_PACKET, n, nbytes, m.F16), m.scratch_required(m.ALGO_ALLPAIR, n, nbytes, m.F16))
    ranks = m.InProcessRanks(n, sb, bulk_scratch_bytes=nbytes + (1 << 20))
    for r in range(n):  # no stale flag word may look like a packet of this call
        m.device_view(ranks.scratch[r].ptr, ranks.scratch_bytes).zero_()
    ins = [torch.rand(count, device="cuda").half() for _ in range(n)]
    outs = [torch.zeros_like(a) for a in ins]
    bulk = algo in (m.ALGO_FULLMESH, m.ALGO_RSAG_ZC)
    arr = ranks.views(ins, outs, bulk=bulk)
    one = (m.RankView * 1)()
    one[0] = arr[0]  # rank 0 only: rank 1's kernel never runs
    nblocks, nthreads = (2, 256) if bulk else (0, 0)
    t0 = time.time()
    rc = m.lib().mscclppAmdAllReduceLaunch(algo, one, 1, n, nbytes, m.F16, m.SUM, nblocks, nthreads, BUDGET_TICKS,
                                           m.stream_ptr())
    assert rc == 0
    torch.cuda.synchronize()  # returns: every wait gave up after its budget
    took = time.time() - t0
    err = ranks.error_details()[0]
    assert err[0] == code, err
    if code == ERR_SEMAPHORE_TIMEOUT:  # detail: channel | peer << 16, rank, tokens seen | wanted << 16
        assert err[1] >> 16 == 1 and err[2] == 0 and (err[3] >> 16) >= 1, err
    else:  # detail: the flag waited for (the first call's), the packet's byte offset, the flag seen there
        # (0: the absent peer never wrote the zeroed slot)
        assert err[1] >= 1 and err[2] < ranks.scratch_bytes and err[3] == 0, err
    assert ranks.errors()[1] == 0  # the absent rank reported nothing
    assert took < 60, took


def _worker(rank, uid, q):
    try:
        import os

        os.environ["MSCCLPP_AMD_SPIN_TIMEOUT_MS"] = "300"
        import torch as th

        import mscclpp_amd as m

        import mp_util

        mp_util.place_rank(rank, 2)
        comm = m.Communicator(rank, 2, uid)
        x = th.ones(512, dtype=th.float16, device="cuda")
        y = th.zeros_like(x)
        comm.all_reduce(x, y, algo="allpair")  # warm: both ranks take part once
        th.cuda.synchronize()
        ok_before = comm.async_error()
        comm.barrier()
        if rank == 0:  # rank 1 never calls this one
            comm.all_reduce(x, y, algo="allpair")
            th.cuda.synchronize()
        after = comm.async_error()
        comm.barrier()
        comm.destroy()
        q.put((rank, (ok_before, after), None))
    except Exception:
        q.put((rank, None, traceback.format_exc()))


def test_absent_peer_reported_by_ncclCommGetAsyncError(built):
    import mscclpp_amd as m

    uid = m.Communicator.unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, uid, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = mp_util.collect(procs, q, 2, 180)
    NCCL_SUCCESS, NCCL_REMOTE_ERROR = 0, 6
    assert got[0] == (NCCL_SUCCESS, NCCL_REMOTE_ERROR), got
    assert got[1] == (NCCL_SUCCESS, NCCL_SUCCESS), got
