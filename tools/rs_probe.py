"""ReduceScatter / AllGather timing and phase split on 2 ranks (processes placed like the tests: a
GPU each where there are two): ncclReduceScatter of a 48 MiB fp16 input per rank, ncclAllGather of
the 24 MiB result, and the AllReduce of the same input for comparison; eager (5 calls) and phase
stamps of one call (PhaseTrace).  -> gpurun_out/rs_probe.json"""
import json
import multiprocessing as mp
import os
import sys
import time
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _t(torch, fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


def worker(rank, n, uid, q):
    try:
        import torch

        import mp_util
        import mscclpp_amd as m

        mp_util.place_rank(rank, n)
        comm = m.Communicator(rank, n, uid)
        S = 48 << 20
        x = torch.rand(S // 2, device="cuda").half()
        rs = torch.empty(S // 2 // n, dtype=torch.float16, device="cuda")
        ag = torch.empty_like(x)
        out = torch.empty_like(x)
        res = {}
        for name, fn in (("allreduce_fullmesh", lambda: comm.all_reduce(x, out, algo="fullmesh")),
                         ("reduce_scatter", lambda: comm.reduce_scatter(x, rs)),
                         ("all_gather", lambda: comm.all_gather(rs, ag))):
            comm.barrier()
            res[name + "_us"] = round(_t(torch, fn), 1)
        for name, fn, ph in (("reduce_scatter", lambda: comm.reduce_scatter(x, rs), "fullmesh"),
                             ("allreduce_fullmesh", lambda: comm.all_reduce(x, out, algo="fullmesh"), "fullmesh")):
            comm.barrier()
            with m.PhaseTrace() as tr:
                fn()
            res[name + "_phases"] = tr.phases(ph)
        comm.barrier()
        comm.destroy()
        q.put((rank, res, None))
    except Exception:
        q.put((rank, None, traceback.format_exc()))


if __name__ == "__main__":
    import mscclpp_amd as m

    n = int(os.environ.get("N", "2"))
    uid = m.Communicator.unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, n, uid, q)) for r in range(n)]
    for p in ps:
        p.start()
    out = {}
    for _ in range(n):
        r, res, err = q.get(timeout=200)
        out[r] = res if err is None else err
    for p in ps:
        p.join(30)
    print(json.dumps(out, indent=1))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", f"rs_probe_n{n}.json"), "w"), indent=1)
