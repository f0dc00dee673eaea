"""Probe: the IB/proxy staging case (buckets start and end in host-pinned memory) with the LL16
self-reduce reading X, Y straight from pinned host memory and writing O straight back (zero-copy
over PCIe, packets in HBM), against copies around a device-resident kernel."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mscclpp_amd as m  # noqa: E402

S = int(os.environ.get("BYTES", 48 << 20))
n = S // 2
dev = torch.device("cuda", 0)
x = torch.rand(n, device=dev).half()
y = torch.rand(n, device=dev).half()
out = torch.empty_like(x)
flags = torch.ones(m.FLAG_SLOTS, dtype=torch.int32, device=dev)
err = torch.zeros(16, dtype=torch.int32, device=dev)
pk = m.DeviceBuffer(2 * S, uncached=True)
hx, hy, ho = (torch.empty(n, dtype=torch.float16).pin_memory() for _ in range(3))
hx.copy_(x.cpu())
hy.copy_(y.cpu())
ref = (x.float() + y.float()).clamp(-65504, 65504).half().cpu()


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def copies():
    x.copy_(hx, non_blocking=True)
    y.copy_(hy, non_blocking=True)
    m.self_reduce_ll16(x, y, pk.ptr, out, flags, err)
    ho.copy_(out, non_blocking=True)


def zero_copy():
    m.self_reduce_ll16(hx, hy, pk.ptr, ho, flags, err)


res = {}
for name, fn in (("copies", copies), ("zero_copy", zero_copy)):
    ho.zero_()
    t = timed(fn)
    res[name] = {"ms": round(t * 1e3, 3), "GBs": round(S / t / 1e9, 2), "correct": bool(torch.equal(ho, ref)),
                 "err": int(err[0].item())}
    print(name, res[name], flush=True)
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open("gpurun_out/staging_probe.json", "w"), indent=1)
