"""Multi-round forms of the 1-GPU LL16 self-reduce (8-48 MiB) by partner placement: the product's
cross-XCD partner workgroup (b ^ 1) against the neighbouring wave of the same workgroup and the
same-XCD workgroup b ^ 8, at skew 0 / 1 / 2, 1024 workgroups of 4 x 1 KiB waves (nt payload),
through tests/bin/libselfreduce_diag.so (mscclppAmdSelfReduceLL16Shape count bits 2 / 3).  Per-launch
time of 20 launches in one HIP graph; every variant checked bit-exactly first.

    python tools/multi_round_probe.py     -> gpurun_out/multi_round_probe.json
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
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


def shape_fn(S, sk, bits, nb=1024, w=4, u=1):
    def f():
        rc = D.mscclppAmdSelfReduceLL16Shape(vp(x.data_ptr()), vp(y.data_ptr()), vp(pk.ptr), vp(out.data_ptr()), S,
                                             vp(flags.data_ptr()), nb, w, u, sk, bits, 500_000_000,
                                             vp(err.data_ptr()), vp(miss.data_ptr()), m.stream_ptr())
        assert rc == 0, (S, sk, bits, rc)
    return f


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


res = {}
for S in [int(v) for v in os.environ.get("SIZES", "8388608,16777216,33554432,50331648").split(",")]:
    xs, ys, os_ = x[: S // 2], y[: S // 2], out[: S // 2]
    variants = {"product": lambda: m.self_reduce_ll16(xs, ys, pk.ptr, os_, flags, err)}
    for sk in (0, 1, 2):
        for pname, bits in (("p1", 0), ("p0", 4), ("p8", 8)):
            variants[f"skew{sk}_{pname}"] = shape_fn(S, sk, bits)
    if os.environ.get("WIDE"):  # 2 KiB per wave, or 8 waves, with the in-workgroup partner
        for sk in (1, 2):
            for nb in (512, 1024):
                variants[f"w4u2_x{nb}_skew{sk}_p0"] = shape_fn(S, sk, 4, nb, 4, 2)
                variants[f"w8u1_x{nb}_skew{sk}_p0"] = shape_fn(S, sk, 4, nb, 8, 1)
    ok = {}
    for k, f in variants.items():
        out.zero_()
        f()
        torch.cuda.synchronize()
        ok[k] = int(err[0].item()) == 0 and torch.equal(out[: S // 2], ref[: S // 2])
        err.zero_()
    times = {k: [] for k in variants}
    for _ in range(3):
        for k, f in variants.items():
            times[k].append(graph_us(f))
    row = {"us": {k: round(float(np.median(v)), 2) for k, v in times.items()}, "correct": ok}
    row["best"] = min(row["us"], key=row["us"].get)
    res[f"{S >> 20}MiB"] = row
    print(json.dumps({f"{S >> 20}MiB": row}), flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(res, open(os.path.join(ROOT, "gpurun_out", "multi_round_probe.json"), "w"), indent=1)
