"""Fabric-free latency of the LL AllReduce kernels (BASELINE configs[3] sizes): n ranks in ONE launch
on one GPU (blockIdx.y = rank, every peer buffer local HBM), fp16, 1 KiB .. 1 MiB, one-hop LL8
(`allpair`, up to ALLPAIR_MAX_KB, default 64) and two-hop LL16 (`packet`), default launch shapes and the alternatives ALLPAIR_SHAPES / PACKET_SHAPES list ("28x512,...").  Time per
call from 20 calls captured in one HIP graph, replayed 10 times (no host launch cost), so what is
left is the kernel's own latency: its dispatch, the packet stores and the polls of each hop.

    python tools/inprocess_ll_probe.py        (writes gpurun_out/inprocess_ll_probe.json)
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mscclpp_amd as m  # noqa: E402

N = int(os.environ.get("NRANKS", 8))
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
sizes = [1 << k for k in range(10, 21)]
def _shapes(var):
    return [(0, 0)] + [tuple(int(v) for v in s.split("x")) for s in os.environ.get(var, "").split(",") if s]


shapes_of = {"allpair": _shapes("ALLPAIR_SHAPES"), "packet": _shapes("PACKET_SHAPES")}
ins_all = [torch.rand(sizes[-1] // 2, device=dev).half() for _ in range(N)]
outs_all = [torch.empty_like(a) for a in ins_all]
sb = max(m.scratch_required(a, N, sizes[-1], m.F16) for a in (m.ALGO_PACKET, m.ALGO_ALLPAIR))
ranks = m.InProcessRanks(N, sb)


def graph_us(fn, calls=20, replays=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(calls):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(replays):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / calls)
    return float(np.median(ts))


rows = []
for algo, name in ((m.ALGO_ALLPAIR, "allpair"), (m.ALGO_PACKET, "packet")):
    for sz in sizes:
        if algo == m.ALGO_ALLPAIR and sz > (int(os.environ.get("ALLPAIR_MAX_KB", 64)) << 10):
            continue
        c = sz // 2
        ins = [a[:c] for a in ins_all]
        outs = [o[:c] for o in outs_all]
        exp = sum(a.float() for a in ins)
        for nb, nt in shapes_of[name]:
            try:
                ranks.all_reduce(ins, outs, algo, nblocks=nb, nthreads=nt)
                torch.cuda.synchronize()
                ok = all(torch.allclose(o.float(), exp, rtol=1e-2, atol=1e-2 * N) for o in outs) and \
                    not any(int(e[0].item()) for e in ranks.err)
                us = graph_us(lambda: ranks.all_reduce(ins, outs, algo, nblocks=nb, nthreads=nt))
                rows.append({"algo": name, "bytes": sz, "shape": f"{nb}x{nt}", "us": round(us, 2), "correct": ok})
            except Exception as e:
                rows.append({"algo": name, "bytes": sz, "shape": f"{nb}x{nt}", "error": str(e)[-120:]})
            print(rows[-1], flush=True)
# the empty-ish floor: a 16-byte copy kernel launch captured the same way
src = torch.zeros(16, dtype=torch.uint8, device=dev)
dst = torch.empty_like(src)
floor = graph_us(lambda: m.lib().mscclppAmdCopy(src.data_ptr(), dst.data_ptr(), 16, 1, m.stream_ptr()))
res = {"nranks": N, "graph_launch_floor_us": round(floor, 2), "rows": rows}
os.makedirs(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out"), exist_ok=True)
json.dump(res, open(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "inprocess_ll_probe.json"), "w"),
          indent=1)
print("floor", floor)
