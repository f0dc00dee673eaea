"""Diagnostic: repeat the in-process mscclpp-test allreduce5 (k5) cases of
tests/test_mscclpp_test_kernels_gpu.py::test_k5_in_place (same parameter order, a fresh
InProcessRanks per case, three calls each) many times and describe any mismatch: which rank, which
chunk (owner) and sub-range (workgroup) it falls in, whether the wrong value equals the un-reduced
input or the sum missing one peer, and whether a second read of the same buffer (after another
synchronize, and through a device-side compare) still sees it -- a stale first copy-out versus a
wrong result in memory."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mscclpp_amd as m  # noqa: E402

CASES = [(2, 4096), (4, 65536), (8, 8192), (8, 1 << 18), (5, 640)]
nb = int(os.environ.get("NB", 24))
reps = int(os.environ.get("REPS", 20))
report = {"reps": reps, "cases_run": 0, "bad_runs": 0, "bad": []}


def describe(n, count, call, r, ins, got, want, again, dev_equal):
    slice_b = count * 4 // n
    blk = ((slice_b + nb - 1) // nb + 15) // 16 * 16
    bad = np.nonzero(got != want)[0]
    i = int(bad[0])
    owner, off = (i * 4) // slice_b, (i * 4) % slice_b
    missing = [p for p in range(n) if (int(want[i]) - int(ins[p][i]) - int(got[i])) % (1 << 32) == 0]
    return {"n": n, "count": count, "call": call, "rank": r, "nbad": int(bad.size), "first": i,
            "last": int(bad[-1]), "owner_chunk": owner, "block": off // blk,
            "owner_chunks": sorted(set(int(b * 4 // slice_b) for b in bad))[:16],
            "got": int(got[i]), "want": int(want[i]), "input_of_rank": int(ins[r][i]),
            "equals_own_input": bool(int(got[i]) == int(ins[r][i])), "equals_sum_missing_rank": missing,
            "second_read_ok": bool(np.array_equal(again, want)), "device_compare_ok": dev_equal}


for rep in range(reps):
    for n, count in CASES:
        ranks = m.InProcessRanks(n, 1 << 16)
        for call in range(3):
            rng = np.random.default_rng(100 + call)
            ins = [rng.integers(-2 ** 31, 2 ** 31, count, dtype=np.int64).astype(np.int32) for _ in range(n)]
            bufs = [torch.from_numpy(a.copy()).cuda() for a in ins]
            ranks.all_reduce(bufs, bufs, m.ALGO_TEST_K5, nblocks=nb, nthreads=512)
            torch.cuda.synchronize()
            report["cases_run"] += 1
            want = np.sum(np.stack([a.astype(np.int64) for a in ins]), axis=0).astype(np.int32)
            bad_any = False
            for r in range(n):
                got = bufs[r].cpu().numpy()
                if np.array_equal(got, want):
                    continue
                bad_any = True
                torch.cuda.synchronize()
                again = bufs[r].cpu().numpy()
                dev_equal = bool(torch.equal(bufs[r], torch.from_numpy(want).cuda()))
                c = describe(n, count, call, r, ins, got, want, again, dev_equal)
                c["rep"], c["errors"] = rep, ranks.errors()
                report["bad"].append(c)
                print(json.dumps(c), flush=True)
            report["bad_runs"] += int(bad_any)
            del bufs
        del ranks
    print(f"rep {rep}: {report['bad_runs']} bad of {report['cases_run']}", flush=True)
os.makedirs("gpurun_out", exist_ok=True)
json.dump(report, open("gpurun_out/k5_diag.json", "w"), indent=1)
print(json.dumps({k: report[k] for k in ("reps", "cases_run", "bad_runs")}))
