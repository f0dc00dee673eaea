"""Summarise a tools/pmc_multirank.sh run (FETCH_SIZE and WRITE_SIZE passes over
tools/inprocess_pmc_run.py: 8 in-process ranks in one launch, so every byte is HBM traffic) into
profiles/<tag>_multirank_pmc.json: per kernel the median bytes per launch against its algorithmic
bytes.  FETCH_SIZE is doubled (gfx950 correction, MI355X_MICROARCH.md §HBM), WRITE_SIZE taken as is.

    python tools/summarize_pmc_multirank.py gpurun_out/pmc_multirank <tag>
"""
import csv
import glob
import json
import os
import statistics
import sys

out_dir, tag = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, MiB = 8, 1 << 20
# algorithmic bytes per launch for all 8 ranks (read, write): zero-copy reads every input once and
# writes every output once (8 S each); fullmesh reads input + peers' scratch regions (8 (S + 7/8 S))
# and writes scratch + own and peers' outputs (the same); LL16 two-hop at S = 1 MiB moves 36 S
KERNELS = {
    "allreduceZeroCopyKernel<0, 0, 8>": ("rsag_zc 32x512, 8 ranks x 48 MiB", 8 * 48 * MiB, 8 * 48 * MiB),
    "allreduceBulkKernel<0, 0, 8, 0, 0>": ("fullmesh 32x512, 8 ranks x 48 MiB", 15 * 48 * MiB, 15 * 48 * MiB),
    "allreduceLL16Kernel<0, 0, 8, 0>": ("packet default shape, 8 ranks x 1 MiB", 36 * MiB, 36 * MiB),
}


def per_launch(key, counter):
    files = glob.glob(os.path.join(out_dir, key, "**", "*counter_collection.csv"), recursive=True)
    got = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"]
            for k in KERNELS:
                if k in name:
                    got.setdefault(k, {}).setdefault(r.get("Dispatch_Id", r.get("Correlation_Id")), 0.0)
                    got[k][r.get("Dispatch_Id", r.get("Correlation_Id"))] += float(r["Counter_Value"])
    return {k: statistics.median(v.values()) * 1024 for k, v in got.items()}


fetch = per_launch("fetch", "FETCH_SIZE")
write = per_launch("write", "WRITE_SIZE")
res = {"note": "8 in-process ranks in one launch on one MI355X; FETCH_SIZE doubled (gfx950 correction, "
               "MI355X_MICROARCH.md), WRITE_SIZE as is; medians over launches", "kernels": {}}
for k, (wl, ar, aw) in KERNELS.items():
    if k in fetch and k in write:
        rd, wr = 2 * fetch[k], write[k]
        res["kernels"][k] = {"workload": wl, "read_bytes": int(rd), "write_bytes": int(wr), "alg_read": ar,
                             "alg_write": aw, "read_ratio": round(rd / ar, 4), "write_ratio": round(wr / aw, 4)}
os.makedirs(os.path.join(root, "profiles"), exist_ok=True)
json.dump(res, open(os.path.join(root, "profiles", f"{tag}_multirank_pmc.json"), "w"), indent=1)
print(json.dumps(res))
