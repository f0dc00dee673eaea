"""GPU tuning sweep for the 1-GPU LL16 self-reduce (fp16 SUM, 48 MiB): variants x grid x packet
memory type, interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24), plus the
streaming-copy HBM ceiling measured in the same run."""
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
L.mscclppAmdSelfReduceLL16Variant.argtypes = [vp, vp, vp, vp, ctypes.c_size_t, vp, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_uint64, vp, vp]
L.mscclppAmdCopy.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int, vp]

S = int(os.environ.get("BYTES", 48 << 20))
n = S // 2
dev = torch.device("cuda", 0)
x = torch.rand(n, device=dev).half()
y = torch.rand(n, device=dev).half()
out = torch.empty_like(x)
flags = torch.ones(m.FLAG_SLOTS, dtype=torch.int32, device=dev)
err = torch.zeros(16, dtype=torch.int32, device=dev)
pk_unc = m.DeviceBuffer(2 * S, uncached=True)
pk_reg = m.DeviceBuffer(2 * S, uncached=False)
ref = (x.float() + y.float()).half()
s = m.stream_ptr()


def run(variant, nb, pk):
    rc = L.mscclppAmdSelfReduceLL16Variant(vp(x.data_ptr()), vp(y.data_ptr()), vp(pk.ptr), vp(out.data_ptr()), S,
                                           vp(flags.data_ptr()), nb, variant, 500_000_000, vp(err.data_ptr()), s)
    assert rc == 0


def timeit(fn, reps=10):
    a = [torch.cuda.Event(enable_timing=True) for _ in range(reps)]
    b = [torch.cuda.Event(enable_timing=True) for _ in range(reps)]
    for i in range(reps):
        a[i].record()
        fn()
        b[i].record()
    torch.cuda.synchronize()
    return [a[i].elapsed_time(b[i]) * 1e3 for i in range(reps)]


configs = []
for pkname, pk in (("uncached", pk_unc), ("regular", pk_reg)):
    for variant in [int(v) for v in os.environ.get('VARIANTS', '0,5,6,10,11,12,13,14,15').split(',')]:
        if pkname == "regular" and variant in (3, 4, 7, 8, 9, 14):
            continue  # nt / plain stores stay in the writer XCD's L2: never visible cross-XCD
        for nb in [int(g) for g in os.environ.get("GRIDS", "256,512,1024").split(",")]:
            configs.append((pkname, pk, variant, nb))
# correctness of every config once
for pkname, pk, variant, nb in configs:
    out.zero_()
    run(variant, nb, pk)
    torch.cuda.synchronize()
    if int(err[0].item()) != 0 or not torch.equal(out, ref):
        print("FAILED", pkname, variant, nb, int(err[0].item()))
        err.zero_()
res = {c[:1] + c[2:]: [] for c in configs}
cp_src = torch.empty(S, dtype=torch.uint8, device=dev)
cp_dst = torch.empty(S, dtype=torch.uint8, device=dev)
copy_t = {nb: [] for nb in (512, 1024, 2048, 4096)}
for rnd in range(5):
    for pkname, pk, variant, nb in configs:
        res[(pkname, variant, nb)] += timeit(lambda: run(variant, nb, pk), 4)
    for nb in copy_t:
        copy_t[nb] += timeit(lambda: L.mscclppAmdCopy(vp(cp_src.data_ptr()), vp(cp_dst.data_ptr()), S, nb, s), 4)
rows = []
for k, v in res.items():
    med = float(np.median(v))
    rows.append({"pk": k[0], "variant": k[1], "nblocks": k[2], "us_med": round(med, 2), "us_min": round(min(v), 2),
                 "TBps_7S": round(7 * S / med / 1e6, 3)})
rows.sort(key=lambda r: r["us_med"])
cp = {nb: {"us_med": round(float(np.median(v)), 2), "TBps_2S": round(2 * S / float(np.median(v)) / 1e6, 3)}
      for nb, v in copy_t.items()}
out_path = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "sweep_self_reduce.json")
json.dump({"rows": rows, "copy": cp}, open(out_path, "w"), indent=1)
for r in rows[:12]:
    print(r)
print("copy", cp)
