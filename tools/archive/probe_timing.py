"""Diagnostic: per-call AllReduce time of one algorithm measured several ways in one process group
(launched by torch.distributed.run).  Separates what the benchmark's timed region adds (host
barrier right before, event pair on the stream, K back-to-back calls) from the kernel itself."""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import mscclpp_amd as m  # noqa: E402

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
ndev = torch.cuda.device_count()
torch.cuda.set_device(rank % ndev)
dist.init_process_group("gloo")
comm = m.Communicator.from_torch_dist()
S = int(os.environ.get("BYTES", 48 << 20))
algo = os.environ.get("ALGO", "rsag_zc")
nb, nt = int(os.environ.get("NB", 128)), int(os.environ.get("NT", 512))
dev = torch.device("cuda", rank % ndev)
x = bench.lcg_tensor(S // 2, rank, 1, torch.float16, dev)
out = torch.empty_like(x)


def call():
    comm.all_reduce(x, out, algo=algo, nblocks=nb, nthreads=nt)


def tmax(v):
    t = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0])


def plain(k, barrier):
    torch.cuda.synchronize()
    if barrier:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(k):
        call()
    torch.cuda.synchronize()
    return tmax((time.perf_counter() - t0) / k) * 1e3


def events(k):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    dist.barrier()
    a.record()
    for _ in range(k):
        call()
    b.record()
    torch.cuda.synchronize()
    return tmax(a.elapsed_time(b) / k)


for _ in range(3):
    call()
res = {}
for rep in range(2):
    for k in (5, 20, 50):
        res[f"plain_k{k}_r{rep}"] = round(plain(k, False), 4)
        res[f"barrier_k{k}_r{rep}"] = round(plain(k, True), 4)
        res[f"events_k{k}_r{rep}"] = round(events(k), 4)
res["graph_per_call"] = round(tmax(bench.graph_time_per_call(call, calls=20, replays=5, sync=dist.barrier)) * 1e3, 4)
if rank == 0:
    print(json.dumps({"algo": algo, "nb": nb, "nt": nt, "ms": res}), flush=True)
comm.destroy()
dist.destroy_process_group()
