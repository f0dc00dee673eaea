"""GPU parity of the DSL executor: n processes (one rank each) on cuda:0 run a JSON execution plan
through mscclppAmdExecutorExecute, call after call; every rank's buffers are compared bit-exactly
with the CPU oracle's simulation of the same plan on the same inputs (oracle/executor_oracle.py,
whose integer results are pinned to exact sums by tests/test_executor_plan.py).  Mirrors the
reference's test_executor (python/test/test_mscclpp.py:657-700): in-place AllReduce of fp16 data,
here with LCG inputs and bit-exact checks instead of a tolerance."""
import json
import multiprocessing as mp
import os
import sys
import traceback

import numpy as np
import mp_util
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PLANS = os.path.join(ROOT, "tests", "golden", "plans")

# (plan, nranks, dtype name, elements per rank, packet type, calls)
CASES_2 = [
    ("allreduce_pkt_n2.json", "f16", 1 << 19, "LL16", 3),
    ("allreduce_pkt_n2.json", "bf16", 1 << 14, "LL8", 2),
    ("allreduce_pkt_n2.json", "f32", 4096, "LL16", 2),
    ("allreduce_rres_n2.json", "f16", 1 << 19, "LL16", 3),
    ("allreduce_put_n2.json", "f32", 1 << 16, "LL16", 3),
]
CASES_4 = [
    ("allreduce_pkt_n4.json", "f16", 1 << 16, "LL16", 3),
    ("allreduce_rres_n4.json", "f32", 1 << 15, "LL16", 2),
    ("allreduce_put_n4.json", "f16", 1 << 14, "LL16", 2),
    ("allreduce_pkt_n4.json", "e4m3", 1 << 16, "LL8", 2),
]
# the reference's own 2-rank plans (test/execution-files, committed as fixtures under plans/ref/):
# the LL packet AllReduce (ppkt / respkt / upkt, double scratch) and the memory-channel AllReduce
# (rres + signal / wait, 16 chunks per rank)
CASES_REF = [
    ("ref/allreduce_packet.json", "f16", 1 << 16, "LL16", 3),
    ("ref/allreduce_packet.json", "bf16", 1 << 12, "LL8", 2),
    ("ref/allreduce_packet.json", "f32", 1 << 14, "LL16", 2),
    ("ref/allreduce.json", "f16", 1 << 19, "LL16", 3),
    ("ref/allreduce.json", "f32", 1 << 16, "LL16", 2),
    # OCP fp8 (execution_kernel.hpp:949-1000: the FP8 kernels, T == AccumT)
    ("ref/allreduce_packet.json", "e4m3", 1 << 16, "LL16", 2),
    ("ref/allreduce.json", "e5m2", 1 << 19, "LL16", 2),
    # uint8 and the software e4m3b15 (execution_kernel.hpp:997-1007), the latter over a uint8 buffer
    ("ref/allreduce_packet.json", "u8", 1 << 16, "LL16", 2),
    ("ref/allreduce_packet.json", "b15", 1 << 16, "LL8", 2),
    ("ref/allreduce.json", "u8", 1 << 19, "LL16", 2),
    ("ref/allreduce.json", "b15", 1 << 19, "LL16", 2),
]
DT = {"f16": 0, "bf16": 1, "f32": 2, "e4m3": 5, "e5m2": 6, "u8": 11, "b15": 12}
NP_VIEW = {"f32": np.int32, "e4m3": np.uint8, "e5m2": np.uint8, "u8": np.uint8, "b15": np.uint8}  # others: 16-bit


def _worker(rank, n, uid, cases, q):
    try:
        os.environ.setdefault("MSCCLPP_AMD_SPIN_TIMEOUT_MS", "5000")
        import torch

        import mscclpp_amd as m
        import oracle_lib as O

        import mp_util

        mp_util.place_rank(rank, n)
        comm = m.Communicator(rank, n, uid)
        ex = m.Executor(comm)
        tdt = {"f16": torch.float16, "bf16": torch.bfloat16, "f32": torch.float32, "e4m3": torch.float8_e4m3fn,
               "e5m2": torch.float8_e5m2, "u8": torch.uint8, "b15": torch.uint8}
        results = []
        for ci, (fname, dt, count, pkt, calls) in enumerate(cases):
            plan = m.ExecutionPlan(os.path.join(PLANS, fname), rank)
            outs = []
            for call in range(calls):
                a = O.lcg(DT[dt], count, rank, 10 * ci + call)
                x = torch.from_numpy(a.view(NP_VIEW.get(dt, np.int16)).copy()).view(tdt[dt]).cuda()
                y = x if plan.is_in_place() else torch.zeros_like(x)
                stream = torch.cuda.current_stream()
                ex.execute(rank, x.data_ptr(), y.data_ptr(), x.numel() * x.element_size(), y.numel() * y.element_size(),
                           m.DataType.float8_e4m3b15 if dt == "b15" else m.EXEC_DTYPES[tdt[dt]], plan, stream,
                           m.PacketType.LL16 if pkt == "LL16" else m.PacketType.LL8)
                torch.cuda.synchronize()
                outs.append(y.cpu().contiguous().view(torch.uint8).numpy().copy())
            err = ex.device_error()
            results.append((fname, dt, outs, err))
            comm.barrier()
        ex.destroy()
        comm.barrier()
        comm.destroy()
        q.put((rank, results, None))
    except Exception:
        q.put((rank, None, traceback.format_exc()))


def _run(n, cases):
    import mscclpp_amd as m

    uid = m.Communicator.unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, n, uid, cases, q)) for r in range(n)]
    for p in procs:
        p.start()
    got = mp_util.collect(procs, q, n, 300)
    return got


def _oracle(n, cases):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import executor_oracle as E
    import oracle_lib as O

    exp = []
    for ci, (fname, dt, count, pkt, calls) in enumerate(cases):
        with open(os.path.join(PLANS, fname)) as f:
            doc = json.load(f)
        eo = E.ExecutorOracle(doc, n)
        per_call = []
        for call in range(calls):
            ins = [O.lcg(DT[dt], count, r, 10 * ci + call).view(np.uint8).copy() for r in range(n)]
            outs = ins if doc["inplace"] else [np.zeros_like(a) for a in ins]
            res = eo.execute(ins, outs, dt, packet=pkt)
            per_call.append([res[r][0 if doc["inplace"] else 1].copy() for r in range(n)])
        exp.append(per_call)
    return exp


def _compare(n, cases, got):
    exp = _oracle(n, cases)
    for rank in range(n):
        for ci, (fname, dt, outs, err) in enumerate(got[rank]):
            assert err == [0, 0, 0, 0], (rank, fname, dt, err)
            for call, o in enumerate(outs):
                e = exp[ci][call][rank]
                bad = np.nonzero(o != e)[0]
                assert bad.size == 0, (rank, fname, dt, call, bad.size, bad[:8])


def test_executor_two_ranks(built):
    _compare(2, CASES_2, _run(2, CASES_2))


def test_executor_four_ranks(built):
    _compare(4, CASES_4, _run(4, CASES_4))


def test_executor_reference_plans(built):
    """The reference's own execution plans, two ranks, bit-exact against the oracle's simulation."""
    _compare(2, CASES_REF, _run(2, CASES_REF))
