"""Probe: how much of the 48 MiB self-reduce's time is HBM vs Infinity Cache, and how the timing
method moves the number.  Per configuration: (1) per-launch event pairs, (2) one event pair around
20 back-to-back launches, (3) 20 launches in one HIP graph, (4) launches each preceded by a 512 MiB
scrub write (cold Infinity Cache; the scrub is timed separately and subtracted).
Packet buffer: uncached (hipDeviceMallocUncached, what bench.py uses) and regular hipMalloc."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mscclpp_amd as m  # noqa: E402

L = m.lib()
vp = ctypes.c_void_p

S = int(os.environ.get("BYTES", 48 << 20))
n = S // 2
dev = torch.device("cuda", 0)
x = torch.rand(n, device=dev).half()
y = torch.rand(n, device=dev).half()
out = torch.empty_like(x)
flags = torch.ones(m.FLAG_SLOTS, dtype=torch.int32, device=dev)
err = torch.zeros(16, dtype=torch.int32, device=dev)
pks = {"uncached": m.DeviceBuffer(2 * S, uncached=True), "regular": m.DeviceBuffer(2 * S, uncached=False)}
ref = (x.float() + y.float()).half()
scrub = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
s = m.stream_ptr()


def sr(pk, variant=0, nb=1024):
    assert L.mscclppAmdSelfReduceLL16Variant(vp(x.data_ptr()), vp(y.data_ptr()), vp(pk.ptr), vp(out.data_ptr()), S,
                                             vp(flags.data_ptr()), nb, variant, 500_000_000, vp(err.data_ptr()), None,
                                             s) == 0


def ev():
    return torch.cuda.Event(enable_timing=True)


def pairs(fn, reps=20):
    es = [(ev(), ev()) for _ in range(reps)]
    for a, b in es:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) * 1e3 for a, b in es]))


def batch(fn, reps=20):
    a, b = ev(), ev()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def graph(fn, reps=20):
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        fn()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    return batch(g.replay, 5) / reps


def cold(fn, reps=10):
    tot, tsc = [], []
    for _ in range(reps):
        a, b, c = ev(), ev(), ev()
        a.record()
        scrub.fill_(1)
        b.record()
        fn()
        c.record()
        torch.cuda.synchronize()
        tot.append(b.elapsed_time(c) * 1e3)
    return float(np.median(tot))


res = {}
for name, pk in pks.items():
    sr(pk)
    torch.cuda.synchronize()
    assert int(err[0].item()) == 0 and torch.equal(out, ref), name
    f = lambda pk=pk: sr(pk)  # noqa: E731
    res[name] = {m_: round(fn(f), 2) for m_, fn in (("pairs", pairs), ("batch", batch), ("graph", graph), ("cold", cold))}
src = torch.empty(S, dtype=torch.uint8, device=dev)
dst = torch.empty(S, dtype=torch.uint8, device=dev)
cp = lambda: L.mscclppAmdCopy(vp(src.data_ptr()), vp(dst.data_ptr()), S, 2048, s)  # noqa: E731
res["copy_S"] = {m_: round(fn(cp), 2) for m_, fn in (("pairs", pairs), ("batch", batch), ("graph", graph), ("cold", cold))}
big = 512 << 20
src2 = torch.empty(big, dtype=torch.uint8, device=dev)
dst2 = torch.empty(big, dtype=torch.uint8, device=dev)
cp2 = lambda: L.mscclppAmdCopy(vp(src2.data_ptr()), vp(dst2.data_ptr()), big, 4096, s)  # noqa: E731
t = batch(cp2, 5)
res["copy_512MiB"] = {"us": round(t, 1), "TBps_2S": round(2 * big / t / 1e6, 3)}
for k, v in res.items():
    if "pairs" in v:
        byt = 7 * S if k in pks else 2 * S
        v["TBps"] = {m_: round(byt / v[m_] / 1e6, 3) for m_ in ("pairs", "batch", "graph", "cold")}
print(json.dumps(res, indent=1))
json.dump(res, open(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "probe_l3.json"), "w"), indent=1)
