"""Ranks on distinct GPUs.  Every rank process sits on device rank % device_count (tests/mp_util.py, as the reference's mp_unit tests place one rank per GPU,
test/mp_unit/mp_unit_tests.cc:109-121), asserts that the ranks' devices differ, and runs the
two-hop LL16, the one-hop LL8 and the zero-copy and fullmesh AllReduce through ncclAllReduce's
communicator, bit-exactly against the CPU oracle.  Every byte between ranks crosses xGMI here:
16-byte {data, flag} packet stores into a peer's scratch, remote loads of peers' inputs, and remote
stores into a peer's output that the owner's next kernel and its copy engine must both see.

On a one-GPU box the same body runs with two ranks sharing the device: every
protocol step and check is the same, only the distinct-device and bus-id assertions need two GPUs,
so the worker is exercised in every GPU test run and the node runs it unedited."""
import multiprocessing as mp
import os
import traceback

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CASES = [("packet", 0, 1 << 18), ("allpair", 0, 4096), ("allpair", 0, 3001), ("rsag_zc", 0, 1 << 20),
         ("fullmesh", 0, 1 << 20), ("fullmesh", 2, 12345), ("auto", 0, 24 << 20)]


def _worker(rank, n, uid, q):
    try:
        os.environ.setdefault("MSCCLPP_AMD_SPIN_TIMEOUT_MS", "10000")
        import torch

        import mp_util
        import mscclpp_amd as m
        import oracle_lib as O

        dev, shared = mp_util.place_rank(rank, n)
        bus = torch.cuda.get_device_properties(dev).pci_bus_id if hasattr(
            torch.cuda.get_device_properties(dev), "pci_bus_id") else dev
        comm = m.Communicator(rank, n, uid)
        tdt = {0: torch.float16, 2: torch.float32}
        bad = []
        for algo, dt, count in CASES:
            ins = [O.lcg(dt, count, r, 5) for r in range(n)]
            x = torch.from_numpy(ins[rank].view(np.int16 if dt < 2 else np.int32).copy()).view(tdt[dt]).cuda()
            y = torch.full_like(x, float("nan"))
            for _ in range(3):
                comm.all_reduce(x, y, algo=None if algo == "auto" else algo)
            torch.cuda.synchronize()
            nbytes = count * (2 if dt < 2 else 4)
            sel = algo if algo != "auto" else \
                {1: "packet", 2: "allpair", 3: "fullmesh", 5: "rsag_zc", 6: "rsag_pipeline"}[
                    m.lib().mscclppAmdSelectAlgo(n, nbytes, dt)]
            if sel == "packet":
                e = O.allreduce_packet(dt, O.SUM, ins, count, 1, max(1 << 22, m.scratch_required(m.ALGO_PACKET, n, nbytes, dt) // 2))[0][rank].view(np.uint8)[:nbytes]
            elif sel == "allpair":
                e = O.allreduce_allpairs(dt, O.SUM, ins, count, 1, max(1 << 22, m.scratch_required(m.ALGO_ALLPAIR, n, nbytes, dt) // 2))[0][rank].view(np.uint8)[:nbytes]
            else:
                sl = ((nbytes + n - 1) // n + 15) // 16 * 16
                nw = (nbytes + 3) // 4
                pad = []
                for a in ins:
                    w = np.zeros(nw, np.uint32)
                    w.view(np.uint8)[:nbytes] = a.view(np.uint8)
                    pad.append(w)
                e = O.allreduce_sliced(dt, O.SUM, pad, nw, sl // 4, 1 if sel == "rsag_zc" else 0)[rank].view(
                    np.uint8)[:nbytes]
            got = y.cpu().contiguous().view(torch.uint8).numpy()
            # read back by a kernel on this GPU too (through its L2), not only by the copy engine
            want = torch.from_numpy(e.copy()).to(y.device)
            same_dev = bool(torch.equal(y.contiguous().view(torch.uint8), want))
            bad.append((algo, dt, count, int(np.count_nonzero(got != e)), same_dev))
        err = comm.device_error()
        comm.destroy()
        q.put((rank, {"dev": dev, "bus": str(bus), "shared": shared, "bad": bad, "err": err}, None))
    except Exception:
        q.put((rank, None, traceback.format_exc()))


def test_ranks_on_distinct_devices_bit_exact(built):
    import mscclpp_amd as m

    n = min(torch.cuda.device_count(), 8) if torch.cuda.device_count() >= 2 else 2
    uid = m.Communicator.unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, n, uid, q)) for r in range(n)]
    for p in procs:
        p.start()
    import mp_util

    got = mp_util.collect(procs, q, n, 300)
    shared = torch.cuda.device_count() < n
    assert shared == (torch.cuda.device_count() < 2)
    if not shared:
        assert len({got[r]["dev"] for r in got}) == n, got
        assert len({got[r]["bus"] for r in got}) == n, got
    for rank, res in got.items():
        assert res["shared"] == shared and res["err"] == 0, (rank, res)
        for algo, dt, count, nbad, same_dev in res["bad"]:
            assert nbad == 0 and same_dev, (rank, algo, dt, count, nbad, same_dev)
