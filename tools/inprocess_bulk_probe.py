"""Fabric-free efficiency of the bulk AllReduce kernels: n ranks in ONE launch on one GPU
(blockIdx.y = rank, every peer buffer local HBM), 48 MiB fp16 per rank, per algorithm and launch
shape.  With no xGMI in the way the kernel's own memory pipeline is what is measured: the HBM rate
of the bytes each algorithm moves (fullmesh / rsag: S(1 + 3(n-1)/n + 1/n) per rank; rsag_zc: 2S;
rsag_pipeline: 2S(1 + 2(n-1)/n)) against the streaming copy of the same run.  A kernel that is slow
here is short of bytes in flight, which the xGMI latency only makes worse.

    python tools/inprocess_bulk_probe.py          (writes gpurun_out/inprocess_bulk_probe.json)
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mscclpp_amd as m  # noqa: E402

N = int(os.environ.get("NRANKS", 8))
S = int(os.environ.get("BYTES", 48 << 20))
count = S // 2
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
ins = [torch.rand(count, device=dev).half() for _ in range(N)]
outs = [torch.empty_like(a) for a in ins]
ref = torch.zeros(count, dtype=torch.float32, device=dev)
ranks = m.InProcessRanks(N, 1 << 20, bulk_scratch_bytes=S + (16 << 20))

HBM = {m.ALGO_FULLMESH: S * (1 + 3 * (N - 1) / N + 1 / N), m.ALGO_RSAG: S * (1 + 3 * (N - 1) / N + 1 / N),
       m.ALGO_RSAG_ZC: 2 * S, m.ALGO_RSAG_PIPELINE: 2 * S * (1 + 2 * (N - 1) / N)}
NAMES = {m.ALGO_FULLMESH: "fullmesh", m.ALGO_RSAG: "rsag", m.ALGO_RSAG_ZC: "rsag_zc",
         m.ALGO_RSAG_PIPELINE: "rsag_pipeline"}
# every rank's grid must be resident at once (cross-rank handshakes): at most 2048 workgroup slots of
# 256 threads would fit at <= 64 VGPRs; kept to 1024 threads per CU: nblocks * N * nthreads <= 256 * 1024
shapes = [(nb, nt) for nb in (8, 16, 32, 64, 128) for nt in (256, 512) if nb * N * nt <= 256 * 1024]
want = [m.ALGO_NAMES[a] for a in os.environ.get("ALGOS", "fullmesh,rsag,rsag_zc,rsag_pipeline").split(",")]
cands = [(a, nb, nt) for a in (m.ALGO_FULLMESH, m.ALGO_RSAG, m.ALGO_RSAG_ZC) if a in want for nb, nt in shapes]
if m.ALGO_RSAG_PIPELINE in want:
    cands += [(m.ALGO_RSAG_PIPELINE, nb, nt) for nb, nt in shapes if 2 * nb * N * nt <= 256 * 1024 and nb >= 2]


def run(a, nb, nt):
    ranks.all_reduce(ins, outs, a, nblocks=nb, nthreads=nt, budget_ticks=300_000_000)


def batch(fn, reps=5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


expect = sum(a.float() for a in ins)  # tolerance check only (bit-exact parity is the tests' job)
rows, ok_c = [], []
for a, nb, nt in cands:
    try:
        for o in outs:
            o.fill_(0)
        run(a, nb, nt)
        torch.cuda.synchronize()
        if any(int(e[0].item()) for e in ranks.err):
            for e in ranks.err:
                e.zero_()
            rows.append({"algo": NAMES[a], "nblocks": nb, "nthreads": nt, "error": "device error word"})
            continue
        good = all(torch.allclose(o.float(), expect, rtol=1e-2, atol=1e-2 * N) for o in outs)
        ok_c.append((a, nb, nt, good))
    except Exception as e:  # a rejected shape
        rows.append({"algo": NAMES[a], "nblocks": nb, "nthreads": nt, "error": str(e)[-120:]})
times = {c[:3]: [] for c in ok_c}
cp_src = torch.empty(S, dtype=torch.uint8, device=dev)
cp_dst = torch.empty(S, dtype=torch.uint8, device=dev)
copy_t = []
for rnd in range(3):
    for c in times:
        times[c].append(batch(lambda: run(*c)))
    copy_t.append(batch(lambda: m.lib().mscclppAmdCopy(ctypes.c_void_p(cp_src.data_ptr()), ctypes.c_void_p(cp_dst.data_ptr()), S, 2048,
                                                     m.stream_ptr())))
for a, nb, nt, good in ok_c:
    us = float(np.median(times[(a, nb, nt)]))
    rows.append({"algo": NAMES[a], "nblocks": nb, "nthreads": nt, "us": round(us, 1), "correct": good,
                 "hbm_TBs": round(N * HBM[a] / us / 1e6, 3), "per_rank_algbw_GBs": round(S / us / 1e3, 1)})
rows.sort(key=lambda r: r.get("us", 1e18))
res = {"nranks": N, "bytes": S, "copy_TBs_2S": round(2 * S / float(np.median(copy_t)) / 1e6, 3), "rows": rows}
os.makedirs(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out"), exist_ok=True)
json.dump(res, open(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", os.environ.get("OUT", "inprocess_bulk_probe.json")), "w"),
          indent=1)
for r in rows:
    print(r)
print("copy TB/s", res["copy_TBs_2S"])
