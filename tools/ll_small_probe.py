"""Small-message LL latency probe (2+ ranks, torch.distributed.run): per-call time of the one-hop
LL8 / two-hop LL16 AllReduce at 1-64 KiB, graph-captured, sizes in forward and reverse order, to
separate first-use effects from size effects.  Diagnostic tool; prints one JSON line on rank 0."""
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import graph_time_per_call  # noqa: E402


def main():
    import mscclpp_amd as m

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", rank)) % torch.cuda.device_count())
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = m.Communicator.from_torch_dist()
    dev = torch.device("cuda", torch.cuda.current_device())
    out = {}
    for order in ("fwd", "rev", "fwd2"):
        kbs = [1, 2, 4, 8, 16, 64]
        if order == "rev":
            kbs = kbs[::-1]
        for algo in ("allpair", "packet"):
            for kb in kbs:
                xs = torch.rand(kb * 512, device=dev).half()
                os_ = torch.empty_like(xs)
                t = graph_time_per_call(lambda: comm.all_reduce(xs, os_, algo=algo), sync=comm.barrier)
                tt = torch.tensor([t], dtype=torch.float64)
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                out[f"{order}:{algo}:{kb}KiB"] = round(float(tt[0]) * 1e6, 2)
    if rank == 0:
        print(json.dumps(out), flush=True)
    comm.destroy()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
