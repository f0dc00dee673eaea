"""torch.distributed ("nccl" backend) running on libmscclpp_amd.so instead of RCCL.

Launch (the reference's test/torch/correctness_test.py flow, with the library interposed the way
its users interpose libmscclpp_nccl.so; TORCH_LIB = the torch wheel's lib/ directory, whose bundled
HIP runtime must be the one this library binds to -- see INTEGRATION.md §1):

    LD_PRELOAD=$TORCH_LIB/libamdhip64.so:$PWD/mscclpp_amd/lib/libmscclpp_amd.so \\
      python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/torch_dist_check.py

Every collective below is checked against a reference computed locally from the same
deterministic per-rank inputs (the LCG of correctness_test.py:44-56): all_reduce (fp16 / bf16 /
fp32, SUM, sizes 1 Ki..4 Mi elements, exact for the order-independent fp32/int cases, the
correctness.py tolerance for fp16/bf16), all_gather_into_tensor, reduce_scatter_tensor,
broadcast and barrier.  Rank 0 prints one JSON line.  Several ranks may share one GPU (RCCL
refuses that, so a passing run on one GPU is itself evidence that the interposed library ran).
"""
import json
import os
import sys

import torch
import torch.distributed as dist

_A, _C, _MASK, _NDIFF = 1664525, 1013904223, 0xFFFFFFFF, 4096


def lcg(n, rank, seq, dtype, device):
    s = (torch.arange(n, device=device, dtype=torch.int64) + rank + seq) & _MASK
    s = (s * _A + _C) & _MASK
    return ((s.remainder(_NDIFF).to(torch.float32)) / float(_NDIFF)).to(dtype)


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    dev = torch.device("cuda", local % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    maps = open("/proc/self/maps").read()
    results = {"interposed": "libmscclpp_amd.so" in maps, "world": world}
    checks = []

    def record(name, ok, err=0.0):
        checks.append({"op": name, "ok": bool(ok), "max_abs_err": float(err)})

    for dtype, tol in ((torch.float32, 0.0), (torch.float16, 5e-3), (torch.bfloat16, 2e-2)):
        for n in (1024, 65536, 1 << 20, 4 << 20):
            for it in range(2):
                x = lcg(n, rank, it, dtype, dev)
                exp = sum(lcg(n, r, it, torch.float32, dev).to(dtype).float() for r in range(world))
                dist.all_reduce(x)
                err = (x.float() - exp).abs().max().item()
                ok = err == 0.0 if tol == 0.0 else err <= tol * max(1.0, exp.abs().max().item())
                record(f"all_reduce {str(dtype)[6:]} {n}", ok, err)
    for n in (4096, 1 << 20):
        inp = lcg(n, rank, 7, torch.float32, dev)
        out = torch.empty(world * n, device=dev)
        dist.all_gather_into_tensor(out, inp)
        exp = torch.cat([lcg(n, r, 7, torch.float32, dev) for r in range(world)])
        record(f"all_gather {n}", torch.equal(out, exp))
        big = lcg(n * world, rank, 9, torch.float32, dev)
        rs = torch.empty(n, device=dev)
        dist.reduce_scatter_tensor(rs, big)
        exp = sum(lcg(n * world, r, 9, torch.float32, dev) for r in range(world)).chunk(world)[rank]
        record(f"reduce_scatter {n}", torch.equal(rs, exp))
    for root in range(world):
        b = lcg(12345, rank, 11, torch.float16, dev)
        dist.broadcast(b, src=root)
        record(f"broadcast root {root}", torch.equal(b, lcg(12345, root, 11, torch.float16, dev)))
    dist.barrier()
    record("barrier", True)
    torch.cuda.synchronize()
    results["checks"] = checks
    results["ok"] = all(c["ok"] for c in checks)
    for c in checks:
        if not c["ok"]:
            print(f"rank {rank} FAILED {c}", file=sys.stderr, flush=True)
    flags = torch.tensor([1 if results["ok"] else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(flags, op=dist.ReduceOp.MIN)  # a 4-byte int32 MIN through the library as well
    results["all_ranks_ok"] = bool(flags.item() == 1)
    print(f"rank {rank} ok={results['ok']} min-reduced flag={flags.item()}", file=sys.stderr, flush=True)
    dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(results), flush=True)
    sys.exit(0 if results["all_ranks_ok"] else 1)


if __name__ == "__main__":
    main()
