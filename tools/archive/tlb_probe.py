"""Probe: does memory re-allocated at the address of a freed allocation receive every store?

For each round: allocate A (kind `first`), write it from every XCD (a torch fill), free it, then
allocate B (kind `second`) of the same size -- normally at the same address -- fill it with a
pattern from every XCD, synchronize, and copy it out.  A store that lands in the old pages (a stale
translation) shows up as words that do not hold the pattern.

    python tools/tlb_probe.py [rounds]        -> gpurun_out/tlb_probe.json
"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mscclpp_amd as m  # noqa: E402


def alloc(kind, nbytes):
    p = ctypes.c_void_p()
    fn = m.lib().mscclppAmdMallocUncached if kind == "uncached" else m.lib().mscclppAmdMalloc
    m.check(fn(ctypes.byref(p), nbytes), "alloc")
    return p.value


def free(ptr):
    m.check(m.lib().mscclppAmdFree(ctypes.c_void_p(ptr)), "free")


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    nbytes = 64 << 20
    out = {}
    for first, second in (("uncached", "coarse"), ("coarse", "coarse"), ("uncached", "uncached"),
                          ("coarse", "uncached")):
        bad_rounds, same_addr, worst = 0, 0, 0
        for r in range(rounds):
            a = alloc(first, nbytes)
            ta = m.device_view(a, nbytes).view(torch.int32)
            ta.fill_(-7)
            torch.cuda.synchronize()
            del ta
            free(a)
            b = alloc(second, nbytes)
            same_addr += int(b == a)
            tb = m.device_view(b, nbytes).view(torch.int32)
            tb.fill_(1000 + r)
            torch.cuda.synchronize()
            nbad = int((tb.cpu() != 1000 + r).sum())
            bad_rounds += int(nbad > 0)
            worst = max(worst, nbad)
            del tb
            free(b)
        out[f"{first}->{second}"] = {"rounds": rounds, "same_address": same_addr, "bad_rounds": bad_rounds,
                                     "worst_bad_words": worst}
        print(f"{first}->{second}", out[f"{first}->{second}"], flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(out, open("gpurun_out/tlb_probe.json", "w"), indent=1)


if __name__ == "__main__" and not os.environ.get("BIG_THEN_SMALL"):
    main()


def big_then_small(gib=8, small=2000):
    """The test suite's pattern: GiB-sized torch tensors written from every XCD, released with
    torch.cuda.empty_cache(), then many small tensors (new 2 MiB segments, often inside the
    released range) filled by a kernel and copied out."""
    big = [torch.empty(1 << 28, dtype=torch.float32, device="cuda") for _ in range(gib)]
    for t in big:
        t.fill_(3.0)
    torch.cuda.synchronize()
    lo = min(t.data_ptr() for t in big)
    hi = max(t.data_ptr() + t.numel() * 4 for t in big)
    del big, t
    torch.cuda.empty_cache()
    bad, inside, keep = 0, 0, []
    for i in range(small):
        x = torch.empty(1 << 18, dtype=torch.int32, device="cuda")
        inside += int(lo <= x.data_ptr() < hi)
        x.fill_(i)
        torch.cuda.synchronize()
        nb = int((x.cpu() != i).sum())
        if nb:
            bad += 1
            print(f"small tensor {i} at {hex(x.data_ptr())}: {nb} words lost", flush=True)
        keep.append(x)  # keep them, so the allocator keeps handing out fresh segments
    return {"small_tensors": small, "inside_released_range": inside, "bad": bad}


if __name__ == "__main__" and os.environ.get("BIG_THEN_SMALL"):
    r = big_then_small()
    print("big_then_small", r, flush=True)
    json.dump(r, open("gpurun_out/tlb_probe_big.json", "w"), indent=1)
