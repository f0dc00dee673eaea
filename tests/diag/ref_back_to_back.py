"""Diagnostic (TEST INFRASTRUCTURE, not collected by pytest): the reference's allreduce2
(python/mscclpp_benchmark/allreduce.cu:225-289, TYPE=int, oracle/_ref) with several calls queued back to
back on every rank stream and no host synchronisation between them -- as the reference's benchmark
times it (allreduce_bench.py bench_time) -- n ranks on one GPU through libref.so's
refBench2RunBackToBack.  Per case: whether the ranks drained, every rank's globalFlag afterwards, and
whether every rank's output equals the sum, for three things run between the calls on each rank stream
(nothing / a no-op kernel over 1024 workgroups / the same kernel invalidating every XCD's L2).  A case
whose ranks do not drain within 3 s is reported and its ranks released by the harness; the run stops
only if they cannot be released.

    python tests/diag/ref_back_to_back.py      (GPU_MAX_HW_QUEUES=16 in the environment)
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import mscclpp_amd as m  # noqa: E402,F401  (the device context and m.device_view)

L = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libref.so"))
vp = ctypes.c_void_p
L.refBench2Open.argtypes = [ctypes.c_char_p, ctypes.c_int]
L.refBench2Open.restype = vp
L.refBench2Close.argtypes = [vp]
L.refMallocUncached.argtypes = [ctypes.c_uint64]
L.refMallocUncached.restype = vp
L.refFree.argtypes = [vp]
L.refBench2RunBackToBack.argtypes = [vp, vp, vp, vp, ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_uint64, ctypes.c_int, vp]
L.refBench2RunBackToBack.restype = ctypes.c_int
L.refBench2Reset.argtypes = [vp, vp, ctypes.c_uint64, ctypes.c_uint64]
L.refBench2Reset.restype = ctypes.c_int
L.refBench2Run.argtypes = [vp, vp, vp, vp, ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_int]
L.refBench2Run.restype = ctypes.c_int
L.refReleaseSpin.argtypes = [vp, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_int]
L.refReleaseSpin.restype = ctypes.c_int
HSACO = os.path.join(ROOT, "oracle", "_ref", "bench_allreduce_int.hsaco")
CALLS = int(os.environ.get("CALLS", 8))
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)


def arr(ps):
    return (ctypes.c_void_p * len(ps))(*ps)


def case(n, words, bpp, threads, between=0):
    sb = 32 * words
    h = L.refBench2Open(HSACO.encode(), n)
    assert h
    scr = [L.refMallocUncached(sb) for _ in range(n)]
    rng = np.random.default_rng(n * 1000 + words)
    ins = [torch.from_numpy(rng.integers(-2 ** 20, 2 ** 20, words).astype(np.int32)).to(dev) for _ in range(n)]
    outs = [torch.zeros_like(x) for x in ins]
    flags = (ctypes.c_uint64 * n)()
    torch.cuda.synchronize()
    try:
        rc = L.refBench2RunBackToBack(h, arr([x.data_ptr() for x in ins]), arr(scr), arr([o.data_ptr() for o in outs]),
                                      words, bpp, threads, CALLS, 3000, sb // 4, between, flags)
        rec = {"n": n, "words": words, "blocks_per_peer": bpp, "threads": threads, "calls": CALLS, "rc": rc,
               "between": ["nothing", "noop_kernel", "l2_invalidate_kernel"][between],
               "globalFlag": list(flags)}
        want = sum(x.long() for x in ins).int()
        if rc == 0:
            rec["outputs_equal_sum"] = all(bool(torch.equal(o, want)) for o in outs)
        elif rc == 2:  # the worker's recovery (tests/ref_kernel_worker.py _run_bench2): reset, one more call
            for o in outs:
                o.zero_()
            torch.cuda.synchronize()
            r1 = L.refBench2Reset(h, arr(scr), sb, 1)
            r2 = L.refBench2Run(h, arr([x.data_ptr() for x in ins]), arr(scr), arr([o.data_ptr() for o in outs]),
                                words, bpp, threads, 3000) if r1 == 0 else -1
            rec["after_reset_rc"] = r2
            if r2 == 0:
                rec["after_reset_outputs_equal_sum"] = all(bool(torch.equal(o, want)) for o in outs)
            elif r2 == 2:  # a second stall: release it as the worker does, then report it as a stop
                rec["after_reset_released"] = any(L.refReleaseSpin(arr(scr), n, sb // 4, v, n, 3000) == 0
                                                  for v in (1, 2, 1))
                rc = 3
        print(json.dumps(rec), flush=True)
        if rc not in (0, 2):  # ranks that could not be released: leave without waiting on them
            print("STOPPED", flush=True)
            os._exit(3)
        return rc
    finally:
        torch.cuda.synchronize()
        L.refBench2Close(h)
        for p in scr:
            L.refFree(p)


# 8 ranks, three variants of what runs between calls on each rank stream (refBench2RunBackToBack):
# nothing, a 1024-workgroup no-op kernel, and the same kernel invalidating every XCD's L2 -- the second
# controls for the third's timing
SHAPES = [(8, 256, 1, 256), (8, 256, 3, 512), (8, 4096, 3, 512), (8, 16384, 3, 512)]
VARIANTS = [int(v) for v in os.environ.get("BETWEEN", "0,2").split(",")]
tally = {}
for between in VARIANTS:
    for n, words, bpp, threads in SHAPES:
        rc = case(n, words, bpp, threads, between)
        tally.setdefault(between, [0, 0])[rc == 2] += 1
print("TALLY " + json.dumps({["nothing", "noop_kernel", "l2_invalidate_kernel"][b]: {"drained": v[0], "stalled": v[1]}
                             for b, v in tally.items()}), flush=True)
print("BACK-TO-BACK DONE", flush=True)
