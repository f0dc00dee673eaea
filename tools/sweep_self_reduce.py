"""GPU sweep of the 1-GPU LL16 self-reduce (BASELINE configs[1], fp16 SUM) by launch shape, 64 KiB ..
48 MiB: the product entry's default shape against alternative (waves per workgroup, KiB per wave and
round, skew, workgroups) shapes of the same kernel template, run through the test diagnostics library
(tests/bin/libselfreduce_diag.so, mscclppAmdSelfReduceLL16Shape).  Per-launch time from 20 launches
captured in one HIP graph (device time, no host launch cost), interleaved rounds in one process;
every shape is checked bit-exactly first.  With COUNT=1 also the first-poll misses per launch.

    python tools/sweep_self_reduce.py            -> gpurun_out/sweep_self_reduce.json
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mscclpp_amd as m  # noqa: E402

vp = ctypes.c_void_p
D = ctypes.CDLL(os.path.join(ROOT, "tests", "bin", "libselfreduce_diag.so"))
D.mscclppAmdSelfReduceLL16Shape.argtypes = [vp, vp, vp, vp, ctypes.c_size_t, vp, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, vp, vp, vp]
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
SMAX = 48 << 20
x = torch.rand(SMAX // 2, device=dev).half()
y = torch.rand(SMAX // 2, device=dev).half()
out = torch.empty_like(x)
flags = torch.ones(m.FLAG_SLOTS, dtype=torch.int32, device=dev)
err = torch.zeros(16, dtype=torch.int32, device=dev)
miss = torch.zeros(4, dtype=torch.int32, device=dev)
pk = m.DeviceBuffer(2 * SMAX)
ref = (x.float() + y.float()).clamp(-65504, 65504).half()


def shape_fn(S, w, u, sk, nb, count=0):
    def f():
        rc = D.mscclppAmdSelfReduceLL16Shape(vp(x.data_ptr()), vp(y.data_ptr()), vp(pk.ptr), vp(out.data_ptr()), S,
                                             vp(flags.data_ptr()), nb, w, u, sk, count, 500_000_000,
                                             vp(err.data_ptr()), vp(miss.data_ptr()), m.stream_ptr())
        assert rc == 0, rc
    return f


def product_fn(S):
    xs, ys, os_ = x[: S // 2], y[: S // 2], out[: S // 2]
    return lambda: m.self_reduce_ll16(xs, ys, pk.ptr, os_, flags, err)


def graph_us(fn, calls=20, replays=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(calls):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(replays):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / (replays * calls)


def default_shape(S):
    w, u, nb, sk = (ctypes.c_int() for _ in range(4))
    m.check(m.lib().mscclppAmdSelfReduceLL16DefaultShape(S, ctypes.byref(w), ctypes.byref(u), ctypes.byref(nb),
                                                         ctypes.byref(sk)), "default shape")
    return w.value, u.value, sk.value, nb.value


def candidates(S):
    """(waves, KiB per wave, skew, workgroups): one round (a workgroup per tile) and two rounds for
    buckets that fit, and 512 / 1024 / 2048 workgroups with the skew from three rounds on."""
    c = []
    for w, u in ((1, 1), (2, 1), (2, 2), (4, 1), (4, 2), (8, 1), (8, 2)):
        tile = w * u * 1024
        tiles = -(-S // tile)
        cap = 1024 * 4 // w  # at most 16 waves per CU
        for nb in sorted({tiles, -(-tiles // 2)} | {g for g in (512, 1024, 2048) if g < tiles}):
            if nb < 2 or nb > cap:
                continue
            rounds = -(-tiles // nb)
            c.append((w, u, 1 if rounds >= 3 else 0, nb))
            if rounds == 1 and w in (4, 8):  # the one-round form with default-policy payload accesses
                c.append((w, u, 0, nb, 2))
            if rounds >= 4 and w == 4:  # partner tiles consumed two rounds late
                c.append((w, u, 2, nb))
    return sorted(set(c))


def name(c):
    return "w%d u%d skew%d x%d" % c[:4] + (" plain" if len(c) > 4 else "")


sizes = [int(v) for v in os.environ.get("SIZES", ",".join(str((64 << 10) << k) for k in range(10))).split(",")] + \
    ([48 << 20] if not os.environ.get("SIZES") else [])
res = {}
for S in sizes:
    cands = candidates(S)
    ok = {}
    for cnd in cands:
        out.zero_()
        shape_fn(S, *cnd)()
        torch.cuda.synchronize()
        ok[cnd] = int(err[0].item()) == 0 and torch.equal(out[: S // 2], ref[: S // 2])
        err.zero_()
    out.zero_()
    product_fn(S)()
    torch.cuda.synchronize()
    prod_ok = torch.equal(out[: S // 2], ref[: S // 2])
    times = {cnd: [] for cnd in cands}
    prod = []
    for _ in range(3):
        prod.append(graph_us(product_fn(S)))
        for cnd in cands:
            times[cnd].append(graph_us(shape_fn(S, *cnd)))
    row = {"default_shape": "w%d u%d skew%d x%d" % default_shape(S), "product_us": round(float(np.median(prod)), 2),
           "product_correct": bool(prod_ok),
           "shapes_us": {name(c): round(float(np.median(t)), 2) for c, t in times.items()},
           "shapes_correct": all(ok.values())}
    best = min(times, key=lambda c: np.median(times[c]))
    row["best"] = name(best)
    row["best_us"] = round(float(np.median(times[best])), 2)
    if os.environ.get("COUNT") or S == 48 << 20:
        misses = {}
        for cnd in cands:
            miss.zero_()
            shape_fn(S, *cnd[:4], (cnd[4] if len(cnd) > 4 else 0) | 1)()  # count bit 0, plain bit 1
            torch.cuda.synchronize()
            misses[name(cnd)] = int(miss[0].item())
        row["first_poll_misses"] = misses
        row["packets"] = S // 8
    res[f"{S >> 10}KiB"] = row
    print(json.dumps({f"{S >> 10}KiB": {k: row[k] for k in ("default_shape", "product_us", "best", "best_us",
                                                             "product_correct", "shapes_correct")}}), flush=True)
res["empty_kernel_graph_us"] = round(graph_us(lambda: torch.cuda._sleep(0)), 2)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(res, open(os.path.join(ROOT, "gpurun_out", "sweep_self_reduce.json"), "w"), indent=1)
