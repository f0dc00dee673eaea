"""Host cost of one AllReduce call (the eager small-message path): 2 ranks on the box's GPU, 1 KiB
fp16, `iters` calls issued back to back; the host time per call is measured around the issuing loop
alone (the device catches up afterwards), for ncclAllReduce (selector + algorithm collection) and for
the explicit-algorithm entry point, plus the same loop with a stream synchronize after every call.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/host_overhead.py
"""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mscclpp_amd as m  # noqa: E402


def main():
    rank = int(os.environ["RANK"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    comm = m.Communicator.from_torch_dist()
    x = torch.rand(512, device="cuda").half()
    y = torch.empty_like(x)
    iters = 2000
    res = {}
    for name, fn in (("ncclAllReduce", lambda: comm.all_reduce(x, y)),
                     ("explicit_allpair", lambda: comm.all_reduce(x, y, algo="allpair")),
                     ("explicit_packet", lambda: comm.all_reduce(x, y, algo="packet"))):
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        dist.barrier()
        t3 = time.perf_counter()
        for _ in range(200):
            fn()
            torch.cuda.synchronize()
        t4 = time.perf_counter()
        res[name] = {"host_us_per_call": round((t1 - t0) / iters * 1e6, 2),
                     "drain_us_per_call": round((t2 - t0) / iters * 1e6, 2),
                     "synced_us_per_call": round((t4 - t3) / 200 * 1e6, 2)}
    if rank == 0:
        print(json.dumps(res))
        os.makedirs("gpurun_out", exist_ok=True)
        json.dump(res, open("gpurun_out/host_overhead.json", "w"), indent=1)
    comm.destroy()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
