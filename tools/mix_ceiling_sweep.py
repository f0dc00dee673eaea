"""How fast can ANY kernel move the self-reduce's 4:3 read:write mix (48 MiB: 4*S read, 3*S
written)?  The generic grid-stride mix kernel (mscclppAmdMixStream) over grids of 256-8192
workgroups, the streaming copy (mscclppAmdCopy) over the same grids, beside the product kernel --
all in one process, interleaved, 20 launches per timing, 5 rounds, medians.
    python tools/mix_ceiling_sweep.py  -> gpurun_out/mix_ceiling_sweep.json"""
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
L = m.lib()
S = 48 << 20
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
x = torch.rand(S // 2, device=dev).half()
y = torch.rand(S // 2, device=dev).half()
out = torch.empty_like(x)
pk = m.DeviceBuffer(2 * S)
pout = torch.empty(2 * S, dtype=torch.uint8, device=dev)
flags = torch.ones(m.FLAG_SLOTS, dtype=torch.int32, device=dev)
err = torch.zeros(16, dtype=torch.int32, device=dev)


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


variants = {"product": lambda: m.self_reduce_ll16(x, y, pk.ptr, out, flags, err)}
for nb in (256, 512, 1024, 2048, 4096, 8192):
    variants[f"mix_{nb}"] = (lambda nb=nb: m.check(L.mscclppAmdMixStream(vp(x.data_ptr()), vp(y.data_ptr()), vp(pk.ptr),
                                                                          vp(pout.data_ptr()), vp(out.data_ptr()), S, nb,
                                                                          m.stream_ptr()), "mix"))
    variants[f"copy_{nb}"] = (lambda nb=nb: m.check(L.mscclppAmdCopy(vp(x.data_ptr()), vp(out.data_ptr()), S, nb,
                                                                      m.stream_ptr()), "copy"))
t = {k: [] for k in variants}
for _ in range(5):
    for k, f in variants.items():
        t[k].append(timed(f))
res = {}
for k, v in t.items():
    us = float(np.median(v))
    nbytes = 7 * S if not k.startswith("copy") else 2 * S
    res[k] = {"us": round(us, 2), "TBs": round(nbytes / us / 1e6, 3)}
res["best_generic_mix"] = max((k for k in res if k.startswith("mix_")), key=lambda k: res[k]["TBs"])
res["product_over_best_generic"] = round(res["product"]["TBs"] / res[res["best_generic_mix"]]["TBs"], 4)
print(json.dumps(res, indent=1))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(res, open(os.path.join(ROOT, "gpurun_out", "mix_ceiling_sweep.json"), "w"), indent=1)
