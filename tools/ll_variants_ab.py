"""Same-process A/B timing of the LL AllReduce kernels' round-3 changes (tests/bin/libll_diag.so,
mscclppAmdDiagAllReduceLL): 8 ranks in one launch on one GPU, fp16 SUM, default launch shapes, per-call
time from 20 calls in one HIP graph, variants interleaved over 5 rounds (box-to-box spread is larger
than the differences measured).  Variant bits switch a part back to its round-2 form: 4 = polls
tested as issued and every peer re-read after a miss, 8 = scalar flag load first, 16 = LL16 polls
all peers at once at every slice size (the product does up to 8192 units per slice), 64 = LL16 step 3
waits on a one-line sentinel before a wave's first pass at every size, 512 = at no size (the product:
from 8192 units per slice).  (Bits 1 and 2, a
batched step 1 / step 3 of LL16, measured slower and were removed; profiles/r3_ll_variants_ab.json
keeps that run.)  Every variant's output is checked against variant 0's.

    python tools/ll_variants_ab.py        -> gpurun_out/ll_variants_ab.json
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

D = ctypes.CDLL(os.path.join(ROOT, "tests", "bin", "libll_diag.so"))
vp = ctypes.c_void_p
D.mscclppAmdDiagAllReduceLL.argtypes = [ctypes.c_int, vp, ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_int, ctypes.c_uint64, vp]
N = 8
torch.cuda.set_device(0)
CASES = [("allpair", kb, (0, 4, 8)) for kb in (1, 4, 16)] + \
        [("packet", kb, (0, 4, 64, 512)) for kb in (1, 16, 128, 256, 512, 1024)]
COUNTED = {"allpair": (0,), "packet": (0, 64, 512)}  # miss counts of these (variant | 32)


def graph_us(fn, calls=20, replays=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
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


res = {}
for algo, kb, variants in CASES:
    code = m.ALGO_NAMES[algo]
    S = kb << 10
    sb = m.scratch_required(code, N, S, m.F16)
    ranks = m.InProcessRanks(N, sb)
    ins = [torch.rand(S // 2, device="cuda").half() for _ in range(N)]
    outs = [torch.empty_like(a) for a in ins]
    arr = ranks.views(ins, outs)

    def call(var):
        def f():
            rc = D.mscclppAmdDiagAllReduceLL(code, arr, N, N, S, 0, 0, var, 500_000_000, m.stream_ptr())
            assert rc == 0, rc
        return f

    call(0)()
    torch.cuda.synchronize()
    ref = [o.clone() for o in outs]
    ok = {}
    for var in variants:
        for o in outs:
            o.zero_()
        call(var)()
        torch.cuda.synchronize()
        ok[var] = all(torch.equal(o, r) for o, r in zip(outs, ref)) and ranks.errors() == [0] * N
    t = {var: [] for var in variants}
    for _ in range(5):
        for var in variants:
            t[var].append(graph_us(call(var)))
    row = {f"v{var}": round(float(np.median(t[var])), 2) for var in variants}
    row["correct"] = all(ok.values())
    # first-poll misses of one call (variant 32: counts into err[8] / err[9] of every rank)
    units = -(-S // 8) // (N if algo == "packet" else 1)  # 8-byte units per slice (LL16) or buffer (LL8)
    polls = N * (N - 1) * units
    for base in COUNTED[algo]:
        key = "first_poll_misses" + (f"_v{base}" if base else "")
        for e in ranks.err:
            e.zero_()
        call(base | 32)()
        torch.cuda.synchronize()
        m8 = sum(int(e[8].item()) for e in ranks.err)
        m9 = sum(int(e[9].item()) for e in ranks.err)
        row[key] = {"reduce": m8, "unpack": m9, "polls_each": polls,
                    "reduce_frac": round(m8 / polls, 4), "unpack_frac": round(m9 / polls, 4)}
        for e in ranks.err:
            e.zero_()
    res[f"{algo}:{kb}KiB"] = row
    print(json.dumps({f"{algo}:{kb}KiB": row}), flush=True)
    del ranks
res["floor_us"] = round(graph_us(lambda: torch.cuda._sleep(0)), 2)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(res, open(os.path.join(ROOT, "gpurun_out", "ll_variants_ab.json"), "w"), indent=1)
