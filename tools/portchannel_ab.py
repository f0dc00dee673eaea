"""A/B of the PortChannel all-to-all (row f1) across library builds, in one GPU session (VERDICT r4
item 3: name the commit behind the round-4 regression).

    python tools/portchannel_ab.py tag=path/to/libmscclpp_amd.so [tag=...] [--rounds 4] [--iters 5]

Each round runs every library once, in a rotating order, as a fresh pair of rank processes (spawn;
both on device 0 of a one-GPU box, as the bench's host_proxy_baseline does).  Every process loads only
its library with ctypes, makes its communicator with that library's own ncclGetUniqueId /
ncclCommInitRank, runs the host-offload loop first (as tools/host_proxy_baseline.py does), then the
three PortChannel modes at 1 MiB per peer `reps` times each.  A library that exports
mscclppAmdPortChannelAllToAllStats also reports each call's per-iteration median / min / max.
Prints one JSON object: per tag and mode, every call's us (rank 0), and their median."""
import argparse
import ctypes
import json
import multiprocessing as mp
import os
import statistics
import sys
import time
import traceback

MODES = ("put+signal", "putWithSignal", "putWithSignalAndFlush")


def worker(rank, n, path, qid, qres, iters, reps, chunk):
    try:
        import torch

        torch.cuda.set_device(rank % max(1, torch.cuda.device_count()))
        L = ctypes.CDLL(path)
        vp, dp = ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)
        uid = ctypes.create_string_buffer(128)
        if rank == 0:
            assert L.ncclGetUniqueId(uid) == 0
            for _ in range(n - 1):
                qid.put(uid.raw)
        else:
            ctypes.memmove(uid, qid.get(timeout=120), 128)

        class Uid(ctypes.Structure):
            _fields_ = [("internal", ctypes.c_char * 128)]

        u = Uid()
        ctypes.memmove(ctypes.addressof(u), uid, 128)
        L.ncclCommInitRank.argtypes = [ctypes.POINTER(vp), ctypes.c_int, Uid, ctypes.c_int]
        comm = vp()
        assert L.ncclCommInitRank(ctypes.byref(comm), n, u, rank) == 0
        L.mscclppAmdHostOffloadAllGather.argtypes = [vp, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, dp]
        o = (ctypes.c_double * 4)()
        assert L.mscclppAmdHostOffloadAllGather(comm, 4096, 10, 10, o) == 0
        res = {"host_offload_graph_us": o[1]}
        stats = hasattr(L, "mscclppAmdPortChannelAllToAllStats")
        if stats:
            L.mscclppAmdPortChannelAllToAllStats.argtypes = [vp, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, dp,
                                                            ctypes.c_int]
        else:
            L.mscclppAmdPortChannelAllToAll.argtypes = [vp, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, dp]
        for mode, name in enumerate(MODES):
            calls = []
            for _ in range(reps):
                o = (ctypes.c_double * 8)()
                t0 = time.perf_counter()
                rc = (L.mscclppAmdPortChannelAllToAllStats(comm, chunk, mode, iters, o, 8) if stats
                      else L.mscclppAmdPortChannelAllToAll(comm, chunk, mode, iters, o))
                wall = time.perf_counter() - t0
                assert rc == 0, rc
                c = {"us": round(o[0], 1), "ok": o[1] == 1.0, "call_ms": round(wall * 1e3, 1)}
                if stats:
                    c.update({"med": round(o[3], 1), "min": round(o[4], 1), "max": round(o[5], 1), "argmax": int(o[6]),
                              "proxy_gap_us": round(o[7], 1)})
                calls.append(c)
            res[name] = calls
        L.ncclCommDestroy.argtypes = [vp]
        L.ncclCommDestroy(comm)
        qres.put((rank, res, None))
    except Exception:  # noqa: BLE001
        qres.put((rank, None, traceback.format_exc()))


def run_pair(path, iters, reps, chunk, n=2, timeout=300, env=None):
    ctx = mp.get_context("spawn")
    saved = dict(os.environ)
    os.environ.update(env or {})  # the spawned ranks inherit it
    qid, qres = ctx.Queue(), ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, n, path, qid, qres, iters, reps, chunk)) for r in range(n)]
    for p in ps:
        p.start()
    os.environ.clear()
    os.environ.update(saved)
    got = {}
    deadline = time.monotonic() + timeout
    try:
        while len(got) < n:
            rank, res, err = qres.get(timeout=max(1.0, deadline - time.monotonic()))
            if err:
                raise RuntimeError(f"rank {rank}: {err}")
            got[rank] = res
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return got[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+", help="tag=path[@VAR=value[,VAR=value]]: a library and its environment")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--chunk", type=int, default=1 << 20)
    a = ap.parse_args()
    libs = []
    for spec in a.libs:
        tag, rest = spec.split("=", 1)
        path, _, envs = rest.partition("@")
        libs.append((tag, path, dict(e.split("=", 1) for e in envs.split(",") if e)))
    out = {tag: {m: [] for m in MODES} | {"host_offload_graph_us": []} for tag, _, _ in libs}
    for r in range(a.rounds):
        order = libs[r % len(libs):] + libs[: r % len(libs)]
        for tag, path, env in order:
            print(f"[ab] round {r} {tag}", file=sys.stderr, flush=True)
            res = run_pair(os.path.abspath(path), a.iters, a.reps, a.chunk, env=env)
            out[tag]["host_offload_graph_us"].append(round(res["host_offload_graph_us"], 2))
            for m in MODES:
                out[tag][m] += res[m]
    summary = {}
    for tag in out:
        summary[tag] = {m: {"median_us": statistics.median(c["us"] for c in out[tag][m]),
                            "calls_over_1ms": sum(c["us"] > 1000 for c in out[tag][m]),
                            "all_ok": all(c["ok"] for c in out[tag][m])} for m in MODES}
        summary[tag]["host_offload_graph_us_median"] = statistics.median(out[tag]["host_offload_graph_us"])
    print(json.dumps({"iters": a.iters, "reps": a.reps, "rounds": a.rounds, "summary": summary, "calls": out}),
          flush=True)


if __name__ == "__main__":
    main()
