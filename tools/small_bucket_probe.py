"""Small-bucket floor of the 1-GPU LL16 self-reduce (BASELINE configs[1] at 64-256 KiB; VERDICT r3
item 5).  Per-call time with 20 calls in one HIP graph, like bench.py's sweep, for the product entry
and for one-round variants of the same kernel (tests/bin/libselfreduce_diag.so,
mscclppAmdSelfReduceSmallProbe): waves per workgroup, partner on another XCD (b ^ 1) or the same XCD
(b ^ 8), packets in uncached (the product's) or cached memory.  Then the phase stamps of one launch
(serialised by the stamps: load -> packet store -> partner ready -> output store -> flags).  Every
variant is checked bit-exactly first.

    python tools/small_bucket_probe.py      -> gpurun_out/small_bucket_probe.json
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
D.mscclppAmdSelfReduceSmallProbe.argtypes = [vp, vp, vp, vp, ctypes.c_size_t, vp, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int, vp, ctypes.c_uint64, vp, vp]
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
SMAX = 4 << 20
x = torch.rand(SMAX // 2, device=dev).half()
y = torch.rand(SMAX // 2, device=dev).half()
out = torch.empty_like(x)
flags = torch.ones(m.FLAG_SLOTS, dtype=torch.int32, device=dev)
err = torch.zeros(16, dtype=torch.int32, device=dev)
pk_uc = m.DeviceBuffer(2 * SMAX)
pk_c = m.DeviceBuffer(2 * SMAX, uncached=False)
trace = torch.zeros(1024 * 8, dtype=torch.int64, device=dev)
ref = (x.float() + y.float()).clamp(-65504, 65504).half()


def probe_fn(S, w, pm, pk, tr=False):
    nb = S // (w * 1024)

    def f():
        rc = D.mscclppAmdSelfReduceSmallProbe(vp(x.data_ptr()), vp(y.data_ptr()), vp(pk.ptr), vp(out.data_ptr()), S,
                                              vp(flags.data_ptr()), nb, w, pm, vp(trace.data_ptr()) if tr else None,
                                              500_000_000, vp(err.data_ptr()), m.stream_ptr())
        assert rc == 0, (S, w, pm, rc)
    return f


def product_fn(S, pk):
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


def correct(fn, S):
    out.zero_()
    fn()
    torch.cuda.synchronize()
    ok = int(err[0].item()) == 0 and torch.equal(out[: S // 2], ref[: S // 2])
    err.zero_()
    return ok


res = {"empty_kernel_graph_us": None}
graph_us(lambda: torch.cuda._sleep(0))  # the first graph of a process runs slow
res["empty_kernel_graph_us"] = round(float(np.median([graph_us(lambda: torch.cuda._sleep(0)) for _ in range(3)])), 2)
SIZES = [int(v) for v in os.environ.get("SIZES", str(64 << 10) + "," + str(128 << 10) + "," + str(256 << 10)).split(",")]
WAVES = [int(v) for v in os.environ.get("WAVES", "1,2,4,8,16").split(",")]
for S in SIZES:
    variants = {"product_uc": product_fn(S, pk_uc), "product_cached": product_fn(S, pk_c)}
    for w in WAVES:
        nb = S // (w * 1024)
        for pm in (0, 1, 8):
            if nb < 1 or (pm == 1 and nb % 2) or (pm == 8 and nb % 16) or (pm == 0 and w < 2) or \
                    (w == 1 and pm == 0) or (w == 16 and pm != 0):
                continue
            for pkn, pk in (("uc", pk_uc), ("cached", pk_c)):
                variants[f"w{w}_x{nb}_p{pm}_{pkn}"] = probe_fn(S, w, pm, pk)
    ok = {k: correct(f, S) for k, f in variants.items()}
    times = {k: [] for k in variants}
    for _ in range(3):
        for k, f in variants.items():
            times[k].append(graph_us(f))
    row = {"us": {k: round(float(np.median(v)), 2) for k, v in times.items()}, "correct": ok}
    row["best"] = min(row["us"], key=row["us"].get)
    # phase stamps of one eager launch (after warm-up), per variant of interest
    phases = {}
    for key, (w, pm, pk) in {} if os.environ.get("NO_PHASES") else {"w4_p1_uc": (4, 1, pk_uc), "w4_p8_uc": (4, 8, pk_uc), "w4_p0_uc": (4, 0, pk_uc),
                             "w8_p0_uc": (8, 0, pk_uc), "w16_p0_uc": (16, 0, pk_uc)}.items():
        nb = S // (w * 1024)
        if pm == 8 and nb % 16:
            continue
        f = probe_fn(S, w, pm, pk, tr=True)
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        trace.zero_()
        f()
        torch.cuda.synchronize()
        t = trace.view(1024, 8)[:nb, :6].cpu().numpy().astype(np.float64)
        d = np.diff(t, axis=1) / 100.0  # 10 ns ticks -> us
        phases[key] = {"load": round(float(d[:, 0].mean()), 2), "pack_store": round(float(d[:, 1].mean()), 2),
                       "partner_ready": round(float(d[:, 2].mean()), 2), "out_store": round(float(d[:, 3].mean()), 2),
                       "flags": round(float(d[:, 4].mean()), 2),
                       "start_spread": round(float((t[:, 0].max() - t[:, 0].min()) / 100.0), 2),
                       "span": round(float((t[:, 5].max() - t[:, 0].min()) / 100.0), 2)}
    row["phases_us"] = phases
    res[f"{S >> 10}KiB"] = row
    print(json.dumps({f"{S >> 10}KiB": {"best": row["best"], "us": row["us"]}}), flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(res, open(os.path.join(ROOT, "gpurun_out", os.environ.get("OUT", "small_bucket_probe.json")), "w"), indent=1)
print(json.dumps(res), flush=True)
