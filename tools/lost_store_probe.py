"""Probe: do this library's allocation patterns leave a later torch buffer that
misses stores?  Each scenario runs the pattern, then allocates torch buffers, fills them with a kernel
(torch fill_) and checks every word twice: copied out (.cpu()) and read through every XCD's L2
(tests/diag/xcd_probe.hip).  A word only some XCDs read wrong is a stale L2 line; a word every XCD
and the copy-out read wrong is missing from memory.

    python tools/lost_store_probe.py [scenario ...]   -> gpurun_out/lost_store_probe.json

Scenarios (the patterns of the long-lived pytest process, one at a time):
  uc_churn        uncached scratch (hipDeviceMallocUncached, 64 KiB .. 1 GiB) allocated, written, freed,
                  many times; torch buffers allocated in between
  big_release_uc  8 x 1 GiB torch tensors written + released (empty_cache), then 8 x 1 GiB uncached
                  buffers written + freed in the same range, then small torch buffers
  big_release_rw  the same with ordinary (cached) hipMalloc buffers in place of the uncached ones
  uc_read_rw      torch buffers read on every XCD, released, the range re-used as uncached memory
                  written by kernels, freed, then re-used by torch and filled
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import diag_lib  # noqa: E402
import mscclpp_amd as m  # noqa: E402

GIB = 1 << 30


def check(tensors, values, label, report):
    """Every tensor t_i (int32) should hold values[i]; record what differs and where."""
    torch.cuda.synchronize()
    bad = []
    for t, v in zip(tensors, values):
        got = t.cpu().numpy()
        n = int((got != v).sum())
        if n:
            want = np.full(t.numel(), v, dtype=np.int32).view(np.uint32)
            bad.append({"ptr": hex(t.data_ptr()), "bytes": t.numel() * 4, "copy_out_bad": n,
                        "per_xcd": diag_lib.xcd_compare(t, want)})
    report.setdefault(label, {"checked_buffers": 0, "bad_buffers": 0, "examples": []})
    r = report[label]
    r["checked_buffers"] += len(tensors)
    r["bad_buffers"] += len(bad)
    r["examples"] = (r["examples"] + bad)[:8]
    return len(bad)


def small_fill_round(k, report, label, count=64, words=1 << 18):
    ts = [torch.empty(words, dtype=torch.int32, device="cuda") for _ in range(count)]
    vals = [1000 * k + i for i in range(count)]
    for t, v in zip(ts, vals):
        t.fill_(v)
    nb = check(ts, vals, label, report)
    return ts, nb


def write_all_xcds(ptr, nbytes, value):
    t = m.device_view(ptr, nbytes).view(torch.int32)
    t.fill_(value)
    s = int(t[:: max(1, t.numel() // 4096)].sum().item())  # read back on many workgroups too
    del t
    return s


def uc_churn(report, rounds=30):
    rng = np.random.default_rng(0)
    keep = []
    for k in range(rounds):
        sz = int(rng.choice([64 << 10, 1 << 20, 16 << 20, 256 << 20, GIB]))
        bufs = [m.DeviceBuffer(sz) for _ in range(int(rng.integers(1, 9)))]
        for i, b in enumerate(bufs):
            write_all_xcds(b.ptr, b.nbytes, 7 + i)
        torch.cuda.synchronize()
        for b in bufs:
            b.free()
        ts, _ = small_fill_round(k, report, "uc_churn")
        keep += ts[: 4]  # some survive, so the caching allocator keeps taking fresh segments
        if k % 10 == 9:
            keep = []
            torch.cuda.empty_cache()
        print(f"uc_churn round {k}: {report['uc_churn']['bad_buffers']} bad so far", flush=True)


def big_release(report, uncached, rounds=3):
    label = "big_release_uc" if uncached else "big_release_rw"
    for k in range(rounds):
        big = [torch.empty(GIB // 4, dtype=torch.float32, device="cuda") for _ in range(8)]
        for t in big:
            t.fill_(3.0)
        s = sum(float(t.sum().item()) for t in big)  # every XCD reads every tensor's lines
        del big, t
        torch.cuda.empty_cache()
        bufs = [m.DeviceBuffer(GIB, uncached=uncached) for _ in range(8)]
        for i, b in enumerate(bufs):
            write_all_xcds(b.ptr, b.nbytes, 11 + i)
        torch.cuda.synchronize()
        for b in bufs:
            b.free()
        for j in range(4):
            ts, _ = small_fill_round(10 * k + j, report, label, count=128)
            del ts
        big2 = [torch.empty(GIB // 4, dtype=torch.int32, device="cuda") for _ in range(8)]
        vals = [500 + i for i in range(8)]
        for t, v in zip(big2, vals):
            t.fill_(v)
        check(big2, vals, label, report)
        del big2
        torch.cuda.empty_cache()
        print(f"{label} round {k}: {report[label]['bad_buffers']} bad so far (sum {s:.0f})", flush=True)


def uc_read_rw(report, rounds=10):
    for k in range(rounds):
        ts = [torch.full((1 << 22,), 5, dtype=torch.int32, device="cuda") for _ in range(64)]
        _ = [int(t.sum().item()) for t in ts]
        del ts, _
        torch.cuda.empty_cache()
        bufs = [m.DeviceBuffer(16 << 20) for _ in range(16)]
        for i, b in enumerate(bufs):
            write_all_xcds(b.ptr, b.nbytes, 21 + i)
        torch.cuda.synchronize()
        for b in bufs:
            b.free()
        ts = [torch.empty(1 << 22, dtype=torch.int32, device="cuda") for _ in range(64)]
        vals = [3000 + 64 * k + i for i in range(64)]
        for t, v in zip(ts, vals):
            t.fill_(v)
        check(ts, vals, "uc_read_rw", report)
        del ts
        torch.cuda.empty_cache()
        print(f"uc_read_rw round {k}: {report['uc_read_rw']['bad_buffers']} bad so far", flush=True)


SCENARIOS = {"uc_churn": uc_churn, "big_release_uc": lambda r: big_release(r, True),
             "big_release_rw": lambda r: big_release(r, False), "uc_read_rw": uc_read_rw}


def main():
    names = sys.argv[1:] or list(SCENARIOS)
    torch.cuda.set_device(0)
    report = {"device": torch.cuda.get_device_name(0)}
    for name in names:
        t0 = time.time()
        SCENARIOS[name](report)
        report.setdefault(name, {})["seconds"] = round(time.time() - t0, 1)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(report, open("gpurun_out/lost_store_probe.json", "w"), indent=1)
    print(json.dumps({k: {kk: vv for kk, vv in v.items() if kk != "examples"} if isinstance(v, dict) else v
                      for k, v in report.items()}), flush=True)


if __name__ == "__main__":
    main()
