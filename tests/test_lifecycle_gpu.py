"""Communicator lifecycle in long-lived processes, two processes placed
by tests/mp_util.py (one per GPU where there are two):

  * create, use and destroy a communicator three times, each cycle growing the LL scratch with a
    forced large LL16 call: the uncached pool's held bytes and the kept imports of the peer's pooled
    blocks stop growing after the first cycle (the blocks come back from the pool and their imports
    are found again, not re-opened);
  * no torch buffer allocated afterwards overlaps a range that ever held an import of the peer's
    uncached memory, and every such buffer receives every store of a kernel, through the copy engine
    and through every XCD's L2 (the lost-store check of tests/test_zz_store_canary_gpu.py);
  * scratch growth needed inside a HIP graph capture fails with ncclInvalidUsage instead of
    synchronizing the device; the same call outside capture grows it, and the capture then works.

Every AllReduce result is compared bit-exactly with the CPU oracle."""
import multiprocessing as mp
import os
import traceback

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N = 2


def _check_packet(O, got, ins, rank, count):
    import mscclpp_amd as m

    half = m.scratch_required(m.ALGO_PACKET, N, count * 2, m.F16) // 2  # the oracle's scratch must hold the call
    exp, _ = O.allreduce_packet(O.F16, O.SUM, ins, count, 1, half)
    return int(np.count_nonzero(got != exp[rank].view(np.uint8)[: count * 2]))


def _log(rank, msg):
    import sys
    import time

    print(f"[lifecycle rank {rank} {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _worker(rank, uids, q):
    try:
        import faulthandler

        faulthandler.dump_traceback_later(120, exit=True)  # a stuck rank says where, then ends
        os.environ.setdefault("MSCCLPP_AMD_SPIN_TIMEOUT_MS", "10000")
        import torch

        import diag_lib
        import mp_util
        import mscclpp_amd as m
        import oracle_lib as O

        mp_util.place_rank(rank, N)
        res = {"cycles": [], "bad": 0}
        # a forced LL16 call on this bucket needs more than the 64 MiB LL scratch made at init
        big = 1 << 20
        while m.scratch_required(m.ALGO_PACKET, N, big * 2, m.F16) <= (64 << 20):
            big *= 2
        res["big_bytes"] = big * 2
        for cycle in range(3):
            _log(rank, f"cycle {cycle}: init")
            comm = m.Communicator(rank, N, uids[cycle])  # a unique id serves one rendezvous
            for algo, count in (("packet", 1 << 16), ("fullmesh", 1 << 20), ("rsag_zc", 12345), ("packet", big)):
                ins = [O.lcg(O.F16, count, r, cycle) for r in range(N)]
                x = torch.from_numpy(ins[rank].view(np.int16).copy()).view(torch.float16).cuda()
                y = torch.zeros_like(x)
                _log(rank, f"cycle {cycle}: {algo} {count}")
                comm.all_reduce(x, y, algo=algo)
                torch.cuda.synchronize()
                got = y.cpu().view(torch.uint8).numpy()
                if algo == "packet":
                    res["bad"] += _check_packet(O, got, ins, rank, count)
                else:
                    res["bad"] += int(np.count_nonzero(got != _sum_bytes(O, ins, algo, rank, count)))
                del x, y
            res["bad"] += comm.device_error()
            _log(rank, f"cycle {cycle}: destroy")
            comm.barrier()
            comm.destroy()
            torch.cuda.empty_cache()
            res["cycles"].append({"pool": m.pool_stats(), "ipc": m.ipc_stats()})
        _log(rank, "cycles done; torch buffers")
        # torch buffers allocated now: none may sit where an import of the peer's uncached memory
        # was, and each must receive every store of a fill kernel
        kept = m.ipc_kept_ranges()
        res["kept"] = len(kept)
        overlaps, lost = 0, []
        bufs = [torch.empty(sz, dtype=torch.int32, device="cuda")
                for sz in [1 << 18] * 32 + [1 << 20] * 8 + [4 << 20] * 4 + [16 << 20] * 2]
        for i, t in enumerate(bufs):
            a, b = t.data_ptr(), t.data_ptr() + t.numel() * 4
            overlaps += sum(1 for base, nb in kept if a < base + nb and base < b)
            t.fill_(9000 + i)
        torch.cuda.synchronize()
        for i, t in enumerate(bufs):
            n_bad = int((t.cpu() != 9000 + i).sum())
            xcd = diag_lib.xcd_compare(t, np.full(t.numel(), 9000 + i, dtype=np.int32).view(np.uint32))
            if n_bad or any(v["bad"] for v in xcd.values()):
                lost.append((hex(t.data_ptr()), n_bad))
        res["overlaps"], res["lost"] = overlaps, lost[:4]
        del bufs
        # growth under capture: refused; eagerly: done; then the capture works and replays exactly
        _log(rank, "capture")
        comm = m.Communicator(rank, N, uids[3])
        count = big
        ins = [O.lcg(O.F16, count, r, 7) for r in range(N)]
        x = torch.from_numpy(ins[rank].view(np.int16).copy()).view(torch.float16).cuda()
        y = torch.zeros_like(x)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        code = None
        with torch.cuda.stream(side):
            side.synchronize()
            g = torch.cuda.CUDAGraph()
            try:
                g.capture_begin()
                try:
                    comm.all_reduce(x, y, algo="packet", stream=side)
                finally:
                    g.capture_end()
            except m.MscclppError as e:
                code = e.code
        res["capture_code"] = code
        del g
        torch.cuda.synchronize()
        comm.all_reduce(x, y, algo="packet")  # grows the scratch, outside capture
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            comm.all_reduce(x, y, algo="packet", stream=side)
        y.zero_()
        torch.cuda.synchronize()
        comm.barrier()
        g.replay()
        torch.cuda.synchronize()
        res["bad_graph"] = _check_packet(O, y.cpu().view(torch.uint8).numpy(), ins, rank, count)
        res["bad"] += comm.device_error()
        comm.barrier()
        del g
        comm.destroy()
        # with no communicator left, the kept imports can be forgotten explicitly (elastic jobs)
        res["released"] = m.ipc_release_kept()
        res["kept_after_release"] = m.ipc_stats()[1]
        q.put((rank, res, None))
    except Exception:
        q.put((rank, None, traceback.format_exc()))


def _sum_bytes(O, ins, algo, rank, count):
    nbytes = count * 2
    sl = ((nbytes + N - 1) // N + 15) // 16 * 16
    nw = (nbytes + 3) // 4
    pad = []
    for a in ins:
        w = np.zeros(nw, np.uint32)
        w.view(np.uint8)[:nbytes] = a.view(np.uint8)
        pad.append(w)
    return O.allreduce_sliced(O.F16, O.SUM, pad, nw, sl // 4, 1 if algo == "rsag_zc" else 0)[rank].view(np.uint8)[:nbytes]


def test_create_destroy_cycles_pool_and_imports_bounded(built):
    import mscclpp_amd as m

    uids = [m.Communicator.unique_id() for _ in range(4)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, uids, q)) for r in range(N)]
    for p in procs:
        p.start()
    import mp_util

    got = mp_util.collect(procs, q, N, 150)
    for rank, res in got.items():
        assert res["bad"] == 0, (rank, res)
        cyc = res["cycles"]
        held = [c["pool"][0] for c in cyc]
        kept = [c["ipc"][1] for c in cyc]
        assert held[0] > 0 and held[1] == held[0] and held[2] == held[0], (rank, cyc)
        assert all(c["pool"][1] == 0 for c in cyc), (rank, cyc)  # nothing of a destroyed comm in use
        # the peer's tokens, LL scratch (grown once per cycle) and bulk scratch: imported once, kept
        assert kept[0] >= 3 and kept[1] == kept[0] and kept[2] == kept[0], (rank, cyc)
        assert res["overlaps"] == 0 and res["lost"] == [], (rank, res)
        assert res["capture_code"] == 5, (rank, res)  # ncclInvalidUsage
        assert res["bad_graph"] == 0, (rank, res)
        assert res["released"] >= kept[0] and res["kept_after_release"] == 0, (rank, res)


def test_uncached_pool_release_during_reuse_drain(built):
    """a block released by another thread while an allocation drains the pool's pending
    list must not be handed out before its own queued work has run.  One thread keeps allocating
    pooled blocks, queuing a delayed fill of 0xAB into each on its own stream and freeing it at once
    (no synchronize); another keeps allocating the same size class and requires every block it gets
    to read back all zero (the pool's zero fill ran after, not before, the previous owner's fill)."""
    import threading

    import torch

    import mscclpp_amd as m

    torch.cuda.set_device(0)
    nbytes, rounds = 1 << 20, 300
    bad, errors = [], []

    def writer():
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                for _ in range(rounds):
                    b = m.DeviceBuffer(nbytes)
                    v = m.device_view(b.ptr, nbytes)
                    torch.cuda._sleep(20000)  # the fill lands well after the free below
                    v.fill_(0xAB)
                    b.free()  # no synchronize: the block goes to the pending list with its fill queued
            s.synchronize()
        except Exception:  # noqa: BLE001
            errors.append(traceback.format_exc())

    def reader():
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                for i in range(rounds):
                    b = m.DeviceBuffer(nbytes)
                    v = m.device_view(b.ptr, nbytes)
                    nz = int(torch.count_nonzero(v).item())
                    if nz:
                        bad.append((i, nz))
                    b.free()
        except Exception:  # noqa: BLE001
            errors.append(traceback.format_exc())

    ts = [threading.Thread(target=writer), threading.Thread(target=reader)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=100)
    torch.cuda.synchronize()
    assert not any(t.is_alive() for t in ts), "pool stress threads did not finish"
    assert not errors, errors[0]
    assert not bad, f"{len(bad)} reused blocks held the previous owner's late fill, first {bad[:3]}"
