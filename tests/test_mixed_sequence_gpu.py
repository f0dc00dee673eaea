"""Back-to-back collectives of every algorithm on one communicator, two processes: a fixed shuffled
sequence of AllReduce calls (LL8, LL16, fullmesh, ring-order RS+AG, zero-copy, pipelined) over
sizes from 1 KiB to 2 MiB, each call on its own input (LCG, seq = call index) and output buffer,
issued without any synchronisation between calls while one rank sleeps before some of them (rank
skew).  The whole sequence is checked bit-exactly against the oracle once the stream drains, so a
call that reads scratch, flags or semaphores still in use by the previous call of another
algorithm -- or a peer's stale input -- shows up as a wrong word (ADVICE r1's pipeline exit race
was of this kind)."""
import multiprocessing as mp
import random
import traceback

import numpy as np
import mp_util
import pytest

pytestmark = pytest.mark.gpu

ALGOS = ["allpair", "packet", "fullmesh", "rsag", "rsag_zc", "rsag_pipeline"]
SIZES = {"allpair": [512, 4096], "packet": [8192, 1 << 17], "fullmesh": [1 << 16, 1 << 20],
         "rsag": [1 << 16, 1 << 20], "rsag_zc": [1 << 16, 1 << 20], "rsag_pipeline": [1 << 16, 1 << 19]}


def _sequence():
    rnd = random.Random(1234)
    seq = [(a, c) for a in ALGOS for c in SIZES[a]] * 2
    rnd.shuffle(seq)
    return seq


def _expected(O, algo, count, ins, rank, n):
    nbytes = count * 2
    if algo == "packet":
        return O.allreduce_packet(O.F16, O.SUM, ins, count, 1, 1 << 24)[0][rank].view(np.uint8)[:nbytes]
    if algo == "allpair":
        return O.allreduce_allpairs(O.F16, O.SUM, ins, count, 1, 1 << 24)[0][rank].view(np.uint8)[:nbytes]
    nw = (nbytes + 3) // 4
    pad = []
    for a in ins:
        w = np.zeros(nw, np.uint32)
        w.view(np.uint8)[:nbytes] = a.view(np.uint8)
        pad.append(w)
    if algo == "rsag_pipeline":
        return None
    sl = ((nbytes + n - 1) // n + 15) // 16 * 16
    return O.allreduce_sliced(O.F16, O.SUM, pad, nw, sl // 4, 1 if algo in ("rsag", "rsag_zc") else 0)[rank].view(
        np.uint8)[:nbytes]


def _worker(rank, n, uid, q):
    try:
        import os
        import time

        os.environ.setdefault("MSCCLPP_AMD_SPIN_TIMEOUT_MS", "8000")
        import torch

        import mp_util
        import mscclpp_amd as m
        import oracle_lib as O

        mp_util.place_rank(rank, n)
        comm = m.Communicator(rank, n, uid)
        seq = _sequence()
        data = []
        for i, (algo, count) in enumerate(seq):
            ins = [O.lcg(O.F16, count, r, 100 + i) for r in range(n)]
            x = torch.from_numpy(ins[rank].view(np.int16).copy()).view(torch.float16).cuda()
            y = torch.full_like(x, float("nan"))
            data.append((ins, x, y))
        torch.cuda.synchronize()
        comm.barrier()
        for i, (algo, count) in enumerate(seq):
            if rank == 1 and i % 3 == 1:
                time.sleep(0.02)  # rank 1 launches late: its peers run ahead by a call
            _, x, y = data[i]
            comm.all_reduce(x, y, algo=algo)
        torch.cuda.synchronize()
        bad = []
        for i, (algo, count) in enumerate(seq):
            ins, _, y = data[i]
            got = y.cpu().contiguous().view(torch.uint8).numpy()
            e = _expected(O, algo, count, ins, rank, n)
            if e is None:
                ref = sum(a.view(np.float16).astype(np.float64) for a in ins)  # lcg gives fp16 bit patterns
                ok = np.allclose(y.float().cpu().numpy(), ref, rtol=2e-3, atol=2e-3)
                nb = 0 if ok else 1
            else:
                nb = int(np.count_nonzero(got != e))
            if nb:
                bad.append((i, algo, count, nb))
        q.put((rank, (bad, comm.device_error()), None))
        comm.barrier()
        comm.destroy()
    except Exception:
        q.put((rank, None, traceback.format_exc()))


@pytest.mark.parametrize("n", [2, 4])
def test_mixed_algorithm_sequence_back_to_back(built, n):
    import mscclpp_amd as m

    uid = m.Communicator.unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, n, uid, q)) for r in range(n)]
    for p in procs:
        p.start()
    got = mp_util.collect(procs, q, n, 240)
    for rank in range(n):
        bad, errc = got[rank]
        assert errc == 0, (rank, errc)
        assert bad == [], (rank, bad)
