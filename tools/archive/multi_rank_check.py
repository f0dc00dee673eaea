"""Diagnostic: N processes (default 8, sharing the box's GPU) run the bench's bit-exact checks for
the bulk and LL algorithms (seq 0, poison, seq 1 -- bench.py check_run) and, on a mismatch,
describe it: how many words, the first bad word, the slice owner it falls in, and what the wrong
value equals -- the poison, the previous call's (seq 0) result, or the sum in another order.

    python tools/multi_rank_check.py [N]       -> gpurun_out/multi_rank_check.json
"""
import json
import os
import sys
import traceback

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

CASES = [("fullmesh", 16, 512), ("fullmesh", 32, 512), ("rsag", 32, 512), ("rsag_zc", 32, 512),
         ("rsag_pipeline", 8, 512), ("rsag_pipeline", 16, 512), ("packet", 0, 0), ("allpair", 0, 0),
         # again, after the pipeline grew the bulk scratch (bench.py's order: tuning, then checks)
         ("fullmesh", 16, 512), ("rsag", 32, 512), ("rsag_zc", 32, 512), ("rsag_pipeline", 8, 512)]
BACK2BACK = int(os.environ.get("BACK2BACK", "0"))  # extra unsynchronised calls before each check
if os.environ.get("PIPELINE_FIRST"):  # the bulk scratch then reaches its final size at the first call
    CASES = CASES[4:6] + CASES[:4] + CASES[6:]
SIZES = {"packet": 1 << 20, "allpair": 16 << 10}
S_BULK = 48 << 20


def expected(O, m, algo, nb, nt, n, ins, S, rank):
    dt = m.F16
    count = S // 2
    if algo in ("packet", "allpair"):
        code = m.ALGO_PACKET if algo == "packet" else m.ALGO_ALLPAIR
        half = m.scratch_required(code, n, S, dt) // 2
        fn = O.allreduce_packet if algo == "packet" else O.allreduce_allpairs
        outs, _ = fn(dt, O.SUM, ins, count, 1, half)
        return outs[rank][: S // 4].copy(), {}
    nw = S // 4
    slice_w = ((S + n - 1) // n + 15) // 16 * 4
    if algo == "rsag_pipeline":
        C = nb * nt * 4
        chunk, order = 4 * C, 1
    else:
        chunk, order = slice_w, (0 if algo == "fullmesh" else 1)
    exp = O.allreduce_owned(dt, O.SUM, ins, nw, n * chunk, chunk, order)[:nw]
    alt = {"other_order": O.allreduce_owned(dt, O.SUM, ins, nw, n * chunk, chunk, 1 - order)[:nw]}
    return exp, alt


def worker(rank, n, uid, q):
    try:
        os.environ.setdefault("MSCCLPP_AMD_SPIN_TIMEOUT_MS", "20000")
        import torch

        import mscclpp_amd as m
        import oracle_lib as O

        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        comm = m.Communicator(rank, n, uid)

        def lcg(count, r, seq):
            i = torch.arange(count, dtype=torch.int64, device=dev)
            s = (i + r + seq) & 0xFFFFFFFF
            s = (s * 1664525 + 1013904223) & 0xFFFFFFFF
            return ((s % 4096).to(torch.float32) / 4096.0).to(torch.float16)

        report = []
        for algo, nb, nt in CASES:
            print(f"rank {rank} case {algo} {nb}x{nt}", file=sys.stderr, flush=True)
            S = SIZES.get(algo, S_BULK)
            a0, a1 = lcg(S // 2, rank, 0), lcg(S // 2, rank, 1)
            o = torch.empty_like(a0)
            for j in range(BACK2BACK):  # back to back, like the bench's tuning and timed loops
                comm.all_reduce(a1 if j % 2 else a0, o, algo=algo, nblocks=nb, nthreads=nt)
            comm.all_reduce(a0, o, algo=algo, nblocks=nb, nthreads=nt)
            torch.cuda.synchronize()
            got0 = o.view(torch.uint8).cpu().numpy().view(np.uint32).copy()
            o.view(torch.int16).fill_(-1)
            comm.all_reduce(a1, o, algo=algo, nblocks=nb, nthreads=nt)
            torch.cuda.synchronize()
            got = o.view(torch.uint8).cpu().numpy().view(np.uint32)
            err = comm.device_error()
            ins1 = [O.lcg(m.F16, S // 2, r, 1) for r in range(n)]
            exp, alt = expected(O, m, algo, nb, nt, n, ins1, S, rank)
            ins0 = [O.lcg(m.F16, S // 2, r, 0) for r in range(n)]
            exp0, _ = expected(O, m, algo, nb, nt, n, ins0, S, rank)
            row = {"algo": algo, "nb": nb, "nt": nt, "rank": rank, "device_error": err,
                   "seq0_ok": bool(np.array_equal(got0, exp0)), "ok": bool(np.array_equal(got, exp))}
            if not row["ok"]:
                bad = np.nonzero(got != exp)[0]
                i = int(bad[0])
                slice_w = ((S + n - 1) // n + 15) // 16 * 4
                row.update({"nbad": int(bad.size), "first": i, "last": int(bad[-1]),
                            "owner_of_first": i // slice_w, "owners": sorted(set((bad // slice_w).tolist()))[:8],
                            "bad_is_poison": int((got[bad] == 0xFFFFFFFF).sum()),
                            "bad_is_seq0": int((got[bad] == exp0[bad]).sum())})
                for k, v in alt.items():
                    row[f"bad_equals_{k}"] = int((got[bad] == v[bad]).sum())
                    row[f"{k}_all_equal"] = bool(np.array_equal(got, v))
            report.append(row)
            del a0, a1, o
        comm.destroy()
        q.put((rank, report, None))
    except Exception:
        q.put((rank, None, traceback.format_exc()))


def main():
    import multiprocessing as mp

    import mscclpp_amd as m

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    uid = m.Communicator.unique_id()
    procs = [ctx.Process(target=worker, args=(r, n, uid, q)) for r in range(n)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(n):
            rank, rep, err = q.get(timeout=600)
            out[rank] = rep if err is None else err
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(out, open("gpurun_out/multi_rank_check.json", "w"), indent=1)
    for r in sorted(out):
        rep = out[r]
        if isinstance(rep, str):
            print(r, rep)
            continue
        for row in rep:
            print(json.dumps(row))


if __name__ == "__main__":
    main()
