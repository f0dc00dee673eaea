"""Worker for test_reference_kernel_gpu.py (run as its own process: it must set GPU_MAX_HW_QUEUES before
HIP starts).  Runs the reference's own allreduce2 (python/mscclpp_benchmark/allreduce.cu:223-289, TYPE=int,
code object built by oracle/build_ref.sh) as n ranks on one GPU through oracle/_ref/libref.so's
refBench2*, three calls per case (flags 1, 2, 3), and the same inputs through this library's k6
(ALGO_TEST_K6) and the CPU oracle's restatement (oracle_mscclpp_test_ll).  Prints one JSON line per case
and "WORKER OK" at the end; any mismatch raises.  TEST INFRASTRUCTURE ONLY."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)

import oracle_lib as O  # noqa: E402

REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref.so")
HSACO = os.path.join(ROOT, "oracle", "_ref", "bench_allreduce_int.hsaco")


def _lib():
    L = ctypes.CDLL(REF_SO)
    vp = ctypes.c_void_p
    L.refBench2Open.argtypes = [ctypes.c_char_p, ctypes.c_int]
    L.refBench2Open.restype = vp
    L.refBench2Close.argtypes = [vp]
    L.refBench2Diag.argtypes = [vp, vp, vp]
    L.refBench2Run.argtypes = [vp, vp, vp, vp, ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    L.refBench2Run.restype = ctypes.c_int
    L.refMallocUncached.argtypes = [ctypes.c_uint64]
    L.refMallocUncached.restype = vp
    L.refFree.argtypes = [vp]
    return L


def _ptrs(ts):
    return (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])


def run_case(L, m, n, count, blocks_per_peer, threads):
    sb = m.scratch_required(m.ALGO_TEST_K6, n, count * 4, m.I32)
    assert sb == 32 * count  # 4 regions of nelems / 2 LL16 packets (allreduce.cu:244-248)
    h = L.refBench2Open(HSACO.encode(), n)
    assert h, "refBench2Open failed"
    ours = m.InProcessRanks(n, sb)
    dev = torch.device("cuda", 0)
    # uncached, as the reference's GpuBuffer allocates packet scratch on AMD (gpu_utils.cc:139-143)
    rptr = [L.refMallocUncached(sb) for _ in range(n)]
    assert all(rptr), "refMallocUncached failed"
    rscr = [m.device_view(p, sb).view(torch.int32) for p in rptr]
    rec = {"n": n, "count": count, "blocks_per_peer": blocks_per_peer, "threads": threads}
    try:
        for call, flag in enumerate((1, 2, 3)):
            rng = np.random.default_rng(1000 * n + 10 * call + count % 997)
            ins = [rng.integers(-2 ** 31, 2 ** 31, count, dtype=np.int64).astype(np.int32) for _ in range(n)]
            dins = [torch.from_numpy(a).to(dev) for a in ins]
            rout = [torch.zeros_like(d) for d in dins]
            torch.cuda.synchronize()
            rc = L.refBench2Run(h, _ptrs(dins), _ptrs(rscr), _ptrs(rout), count, blocks_per_peer, threads, 20000)
            if rc == 2:  # ranks still spinning: say which and with what flag, then leave without waiting
                done, flags = (ctypes.c_int * n)(), (ctypes.c_uint64 * n)()
                drc = L.refBench2Diag(h, done, flags)
                print(json.dumps({"timeout": rec, "call": call, "diag_rc": drc, "done": list(done),
                                  "globalFlag": list(flags)}), flush=True)
                import subprocess
                ps = subprocess.run(["ps", "-eo", "pid,ppid,etimes,stat,cmd"], stdout=subprocess.PIPE, text=True)
                print("\n".join(x[:200] for x in ps.stdout.splitlines() if "python" in x or "PID" in x), flush=True)
                os._exit(3)
            assert rc == 0, f"refBench2Run returned {rc}"
            douts = [torch.zeros_like(d) for d in dins]
            ours.all_reduce(dins, douts, m.ALGO_TEST_K6)
            torch.cuda.synchronize()
            assert ours.errors() == [0] * n
            exp, scr = O.mscclpp_test_ll([a.view(np.uint32) for a in ins], count, flag, sb)
            want = np.sum(np.stack([a.astype(np.int64) for a in ins]), axis=0).astype(np.uint32)
            for r in range(n):
                ref_out = rout[r].cpu().numpy().view(np.uint32)
                our_out = douts[r].cpu().numpy().view(np.uint32)
                assert np.array_equal(ref_out, want), f"reference output, rank {r}, call {call}"
                assert np.array_equal(exp[r], ref_out), f"oracle vs reference output, rank {r}, call {call}"
                assert np.array_equal(our_out, ref_out), f"k6 vs reference output, rank {r}, call {call}"
            if call == 0:  # fresh scratch: the whole packet image is a function of the inputs and flag 1
                for r in range(n):
                    ref_img = rscr[r].cpu().numpy().view(np.uint32)
                    our_img = ours.scratch_tensor(r, sb).cpu().numpy().view(np.uint32)
                    assert np.array_equal(scr[r], ref_img), f"oracle vs reference scratch image, rank {r}"
                    assert np.array_equal(our_img, ref_img), f"k6 vs reference scratch image, rank {r}"
                rec["scratch_words_compared"] = int(n * sb // 4)
        rec["calls"] = 3
    finally:
        torch.cuda.synchronize()
        L.refBench2Close(h)
        for p in rptr:
            L.refFree(p)
    return rec


def main():
    cases = json.loads(sys.argv[1])
    import mscclpp_amd as m

    torch.cuda.set_device(0)
    L = _lib()
    for n, count, bpp, threads in cases:
        print(json.dumps(run_case(L, m, n, count, bpp, threads)), flush=True)
    print("WORKER OK", flush=True)


if __name__ == "__main__":
    main()
