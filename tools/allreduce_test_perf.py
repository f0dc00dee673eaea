"""allreduce_test_perf -- the mscclpp-test AllReduce harness restated on libmscclpp_amd.so.

Reference: test/mscclpp-test/common.cc (options :547-620, benchTime :202-227, runTest :231-328,
checkData :346-360) and allreduce_test.cu (runColl :1107-1170, initData :1172-1183, getBw
:1185-1190).  One process per GPU, launched like the benchmark:

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        tools/allreduce_test_perf.py -b 24K -e 48M -f 2 -k 6 -o perf.jsonl

Kernels (-k): 1, 2, 5, 6, 7 -- the harness's own int32 kernels (allreduce1 ring through the host proxy,
allreduce2 LL16 one-hop on one node, allreduce5 AMD branch, allreduce6 LL16, allreduce7 LL8); or a product algorithm name (packet, allpair, fullmesh,
rsag, rsag_zc) run on the same int32 data.  Timing is the reference's: `iters` calls captured in one
HIP graph, the graph launched `-G` times after a barrier, time / iters / launches, averaged over
ranks (-a 1); data check = the known answer input = rank -> n(n-1)/2 on every element.  Rows are
printed in the reference's table and, with -o, appended as JSON lines with the reference's keys
(name, kernel, ranks, ranksPerNode, size, time, algBw, busBw; common.cc:301-312).
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

IN_PLACE = {"1": True, "2": False, "5": True, "6": False, "7": False}  # isInPlace (allreduce_test.cu:1262-1264)


def parse_size(v):
    """common.cc parseSize: an optional K/M/G suffix (powers of 1024)."""
    v = v.strip()
    mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}.get(v[-1].upper(), 1)
    return int(float(v[:-1] if mult > 1 else v) * mult)


def parse():
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("-b", "--minbytes", type=parse_size, default=32 << 20)
    p.add_argument("-e", "--maxbytes", type=parse_size, default=32 << 20)
    p.add_argument("-i", "--stepbytes", type=parse_size, default=1 << 20)
    p.add_argument("-f", "--stepfactor", type=int, default=1)
    p.add_argument("-n", "--iters", type=int, default=20)
    p.add_argument("-w", "--warmup_iters", type=int, default=10)
    p.add_argument("-c", "--check", type=int, default=1)
    p.add_argument("-G", "--cudagraph", type=int, default=15, help="graph launches per size")
    p.add_argument("-a", "--average", type=int, default=1, help="0 rank 0, 1 mean, 2 min, 3 max over ranks")
    p.add_argument("-k", "--kernel_num", default="6")
    p.add_argument("-o", "--output_file", default="")
    return p.parse_args()


def sizes(a):
    s = a.minbytes
    while s <= a.maxbytes:
        yield s
        s = s * a.stepfactor if a.stepfactor > 1 else s + a.stepbytes


def run_k1(a, m, comm, rank, world):
    """-k 1: each size runs mscclppAmdProxyRingAllReduce (setup, data check, graph timing inside)."""
    errors = 0
    if rank == 0:
        print("#       size         count     time   algbw   busbw  #wrong   (allreduce1: ring via host proxy)",
              flush=True)
    for size in sizes(a):
        count = size // 4
        us, ok, _ = comm.proxy_ring_all_reduce(count, a.iters, a.cudagraph)
        t = torch.tensor([us], dtype=torch.float64)
        dist.all_reduce(t)
        us = float(t[0]) / world
        ok_t = torch.tensor([0 if ok else 1], dtype=torch.int64)
        dist.all_reduce(ok_t)
        errors += int(ok_t[0])
        alg = size / 1e3 / us
        bus = alg * 2 * (world - 1) / world
        if rank == 0:
            print(f"{size:12d}  {count:12d}  {us:7.1f}  {alg:6.2f}  {bus:6.2f}  {int(ok_t[0]):5d}", flush=True)
            if a.output_file:
                with open(a.output_file, "a") as f:
                    f.write(json.dumps({"name": "allreduce", "kernel": "1", "ranks": world, "ranksPerNode": world,
                                        "size": size, "time": us, "algBw": alg, "busBw": bus}) + "\n")
    if rank == 0:
        print(f"# Out of bounds values : {errors} {'OK' if errors == 0 else 'FAILED'}", flush=True)
    comm.destroy()
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(1 if errors else 0)


def main():
    a = parse()
    import mscclpp_amd as m

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    ndev = torch.cuda.device_count()
    torch.cuda.set_device(local % ndev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = m.Communicator.from_torch_dist()
    kname = a.kernel_num
    algo = None if kname == "1" else (m.ALGO_NAMES["k" + kname] if kname in IN_PLACE else m.ALGO_NAMES[kname])
    in_place = IN_PLACE.get(kname, False)
    dev = torch.device("cuda", local % ndev)
    maxc = a.maxbytes // 4
    inp = torch.zeros(maxc, dtype=torch.int32, device=dev)
    res = inp if in_place else torch.zeros(maxc, dtype=torch.int32, device=dev)
    expected = world * (world - 1) // 2
    stream = torch.cuda.current_stream()

    def run(count):
        comm.all_reduce(inp[:count], res[:count], algo=algo)

    def init(count):
        inp[:count].fill_(rank)  # initData: input = rank (allreduce_test.cu:1172-1177)
        torch.cuda.synchronize()

    def reduce_time(v):
        t = torch.tensor([v], dtype=torch.float64)
        if a.average == 0:
            dist.broadcast(t, 0)
            return float(t[0])
        op = {1: dist.ReduceOp.SUM, 2: dist.ReduceOp.MIN, 3: dist.ReduceOp.MAX, 4: dist.ReduceOp.SUM}[a.average]
        dist.all_reduce(t, op=op)
        return float(t[0]) / (world if a.average == 1 else 1)

    if kname == "1":  # allreduce1: the proxy-driven ring owns its buffers, channels and proxy thread
        return run_k1(a, m, comm, rank, world)
    # warm-up at the largest and the smallest size (runTest :232-250)
    for sz in (a.maxbytes, a.minbytes):
        for _ in range(a.warmup_iters):
            run(sz // 4)
        torch.cuda.synchronize()
        comm.barrier()
    if rank == 0:
        print("#\n#                                        in-place                       out-of-place")
        print("#       size         count     time   algbw   busbw  #wrong     time   algbw   busbw  #wrong")
        print("#        (B)    (elements)     (us)  (GB/s)  (GB/s)             (us)  (GB/s)  (GB/s)", flush=True)
    errors_total = 0
    for size in sizes(a):
        count = size // 4
        init(count)
        # benchTime (:202-227): iters calls in one graph, launched -G times after a barrier
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=torch.cuda.Stream()):
            for _ in range(a.iters):
                run(count)
        torch.cuda.synchronize()
        comm.barrier()
        t0 = time.perf_counter()
        for _ in range(a.cudagraph):
            g.replay()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.iters / a.cudagraph
        dt = reduce_time(dt)
        del g
        nerr = 0
        if a.check:
            init(count)
            comm.barrier()
            run(count)
            torch.cuda.synchronize()
            nerr = int((res[:count] != expected).sum().item())
            t = torch.tensor([nerr], dtype=torch.int64)
            dist.all_reduce(t)
            nerr = int(t[0])
            errors_total += nerr
        us = dt * 1e6
        alg = size / 1e9 / dt
        bus = alg * 2 * (world - 1) / world
        if rank == 0:
            ts = f"{us:7.0f}" if us >= 10000 else (f"{us:7.1f}" if us >= 100 else f"{us:7.2f}")
            pad = "" if in_place else " " * 33
            print(f"{size:12d}  {count:12d}{pad}  {ts}  {alg:6.2f}  {bus:6.2f}  {nerr:5d}", flush=True)
            if a.output_file:
                with open(a.output_file, "a") as f:
                    f.write(json.dumps({"name": "allreduce", "kernel": kname, "ranks": world,
                                        "ranksPerNode": world, "size": size, "time": us, "algBw": alg,
                                        "busBw": bus}) + "\n")
    if rank == 0:
        print(f"# Out of bounds values : {errors_total} {'OK' if errors_total == 0 else 'FAILED'}", flush=True)
    comm.destroy()
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(1 if errors_total else 0)


if __name__ == "__main__":
    main()
