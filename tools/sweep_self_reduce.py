"""GPU tuning sweep for the 1-GPU LL16 self-reduce (fp16 SUM, 48 MiB): kernel variants x grid,
interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24), the first-poll miss count
of the skewed and unskewed forms (variants 4 / 5), and the streaming-copy HBM ceiling measured in
the same run.  Variants: mscclppAmdSelfReduceLL16Variant in include/mscclpp_amd/mscclpp_amd.h."""
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
miss = torch.zeros(4, dtype=torch.int32, device=dev)
pk = m.DeviceBuffer(2 * S, uncached=True)
ref = (x.float() + y.float()).clamp(-65504, 65504).half()
s = m.stream_ptr()


def run(variant, nb):
    rc = L.mscclppAmdSelfReduceLL16Variant(vp(x.data_ptr()), vp(y.data_ptr()), vp(pk.ptr), vp(out.data_ptr()), S,
                                           vp(flags.data_ptr()), nb, variant, 500_000_000, vp(err.data_ptr()),
                                           vp(miss.data_ptr()), s)
    assert rc == 0


def batch(fn, reps=10):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


variants = [int(v) for v in os.environ.get("VARIANTS", "0,1,2,3").split(",")]
grids = [int(g) for g in os.environ.get("GRIDS", "512,1024").split(",")]
configs = [(v, nb) for v in variants for nb in grids]
for v, nb in configs:  # correctness of every config once
    out.zero_()
    run(v, nb)
    torch.cuda.synchronize()
    if int(err[0].item()) != 0 or not torch.equal(out, ref):
        print("FAILED", v, nb, int(err[0].item()))
        err.zero_()
# first-poll misses per launch (packets; each miss re-reads a 16-byte packet at least once)
misses = {}
for v, name in ((4, "skewed"), (5, "unskewed")):
    vals = []
    for _ in range(5):
        miss.zero_()
        run(v, 1024)
        torch.cuda.synchronize()
        vals.append(int(miss[0].item()))
    misses[name] = {"packets_per_launch_median": int(np.median(vals)),
                    "bytes_per_launch_median": int(np.median(vals)) * 16, "of_packets": S // 8}
res = {c: [] for c in configs}
cp_src = torch.empty(S, dtype=torch.uint8, device=dev)
cp_dst = torch.empty(S, dtype=torch.uint8, device=dev)
copy_t = {nb: [] for nb in (1024, 2048, 4096)}
for rnd in range(5):
    for v, nb in configs:
        res[(v, nb)].append(batch(lambda: run(v, nb), 10))
    for nb in copy_t:
        copy_t[nb].append(batch(lambda: L.mscclppAmdCopy(vp(cp_src.data_ptr()), vp(cp_dst.data_ptr()), S, nb, s), 10))
rows = []
for (v, nb), t in res.items():
    med = float(np.median(t))
    rows.append({"variant": v, "nblocks": nb, "us_med": round(med, 2), "us_min": round(min(t), 2),
                 "TBps_7S": round(7 * S / med / 1e6, 3)})
rows.sort(key=lambda r: r["us_med"])
cp = {nb: {"us_med": round(float(np.median(t)), 2), "TBps_2S": round(2 * S / float(np.median(t)) / 1e6, 3)}
      for nb, t in copy_t.items()}
os.makedirs(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out"), exist_ok=True)
out_path = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "sweep_self_reduce.json")
json.dump({"rows": rows, "copy": cp, "first_poll_misses": misses}, open(out_path, "w"), indent=1)
for r in rows:
    print(r)
print("copy", cp)
print("misses", misses)
