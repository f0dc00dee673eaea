"""Diagnostic: N processes on cuda:0 through the NCCL ABI, with progress printed per phase."""
import multiprocessing as mp
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def log(rank, msg):
    print(f"[{time.strftime('%H:%M:%S')}] rank {rank}: {msg}", file=sys.stderr, flush=True)


def worker(rank, n, uid, algos):
    os.environ.setdefault("MSCCLPP_AMD_SPIN_TIMEOUT_MS", "3000")
    log(rank, "importing torch")
    import torch

    import mscclpp_amd as m

    torch.cuda.set_device(0)
    torch.zeros(1, device="cuda")
    log(rank, "ncclCommInitRank")
    comm = m.Communicator(rank, n, uid)
    log(rank, "comm ready")
    for algo in algos:
        for count in (4096, 1 << 16, 1 << 20):
            x = torch.full((count,), float(rank + 1), dtype=torch.float16, device="cuda")
            out = torch.zeros_like(x)
            comm.all_reduce(x, out, algo=algo)
            torch.cuda.synchronize()
            e = comm.device_error()
            ok = bool(torch.all(out == n * (n + 1) / 2))
            log(rank, f"{algo} count={count} err={e} ok={ok}")
    comm.barrier()
    comm.destroy()
    log(rank, "done")


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    algos = sys.argv[2].split(",") if len(sys.argv) > 2 else ["allpair", "packet", "fullmesh"]
    import mscclpp_amd as m

    uid = m.Communicator.unique_id()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=worker, args=(r, n, uid, algos)) for r in range(n)]
    for p in ps:
        p.start()
    for p in ps:
        p.join()
    print("exit codes", [p.exitcode for p in ps], flush=True)
