"""mscclpp_amd benchmark (driver contract: one JSON line on rank 0).

N = 1  -> BASELINE.json configs[1]: the 1-GPU LL16 pack + sum + unpack self-reduce, fp16, 48 MiB,
          device-resident (the HBM-roofline check of the LL hot path).
N > 1  -> BASELINE.json configs[2]: ncclAllReduce of a 48 MiB fp16 bucket (2048 x 12288, the
          README's GPT-3 TP bucket) per rank, one process per GPU, one-sided puts over xGMI
          through libmscclpp_amd.so (no RCCL underneath).  Launched by torch.distributed.run.

value = algbw = S / t (GB/s): S = bucket bytes per rank, t = max over ranks of the time per step
inside the timed region (barrier + synchronize on both sides).  Inputs are resident in HBM before
the timed region starts.  The roofline object prices the dominant kernel with its live HIP-event
duration; cpu_baseline times the CPU oracle (oracle/liboracle.so) on a bounded sample.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
XGMI_LINK_GBS = 153.6          # per link, task-stated


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--bytes", type=int, default=48 << 20)
    p.add_argument("--algo", default=None,
                   help="force an AllReduce algorithm (N>1): packet|allpair|fullmesh|rsag|rsag_zc|rsag_pipeline")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-extras", action="store_true", help="N>1: skip the LL latency sweep and the fp32 1 GiB run")
    return p.parse_args()


def cpu_baseline_self_reduce(nbytes, budget_s):
    """Oracle (scalar C port, 1 thread) pack+sum+unpack on the same workload, bounded in time."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O

    count = nbytes // 2
    x = O.lcg(O.F16, count, 0, 0)
    y = O.lcg(O.F16, count, 1, 0)
    iters, t0 = 0, time.perf_counter()
    while True:
        O.self_reduce(O.F16, O.SUM, x, y, iters + 1)
        iters += 1
        el = time.perf_counter() - t0
        if el >= budget_s or iters >= 200:
            break
    return {"value": round(nbytes * iters / el / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": f"{iters} x oracle_self_reduce fp16 {nbytes >> 20} MiB (scalar C, 1 thread) in {el:.1f} s"}


def cpu_baseline_allreduce(nbytes, n, budget_s):
    """Oracle fullmesh-order AllReduce arithmetic for n ranks on a bounded slice of the bucket."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O

    sample = min(nbytes, 8 << 20)
    count = sample // 2
    ins = [O.lcg(O.F16, count, r, 0).view(np.uint32) for r in range(n)]
    nw = sample // 4
    iters, t0 = 0, time.perf_counter()
    while True:
        O.allreduce_sliced(O.F16, O.SUM, ins, nw, nw // n, 0)
        iters += 1
        el = time.perf_counter() - t0
        if el >= budget_s or iters >= 1000:
            break
    return {"value": round(sample * iters / el / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": f"{iters} x oracle {n}-rank fullmesh-order fp16 sum of {sample >> 20} MiB (scalar C, 1 thread)"}


def committed_traffic(S):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/<tag>_self_reduce_pmc.json:
    2*FETCH_SIZE + WRITE_SIZE, the gfx950 correction of MI355X_MICROARCH.md §HBM), or None."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_self_reduce_pmc.json")))
    if not files or S != 48 << 20:
        return None
    d = json.load(open(files[-1]))
    return d.get("hbm_bytes_per_launch_corrected")


def host_proxy_baseline():
    """BASELINE config 1 (host-proxy path, 2 ranks, 4 KiB) -- spawned before this process touches the GPU."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    try:
        import host_proxy_baseline as H

        return H.run(2, 4096, timeout=240)
    except Exception as e:  # recorded, never fatal for the headline line
        return {"error": str(e)[-400:]}


def staged_rate(m, S, x, y, out, pk, flags, err, reps=10):
    """IB/proxy staging: buckets start and end in host-pinned memory, so time H2D(x, y) + kernel + D2H(out)."""
    hx = torch.empty(x.numel(), dtype=x.dtype).pin_memory()
    hy = torch.empty_like(hx).pin_memory()
    ho = torch.empty_like(hx).pin_memory()
    hx.copy_(x.cpu())
    hy.copy_(y.cpu())

    def step():
        x.copy_(hx, non_blocking=True)
        y.copy_(hy, non_blocking=True)
        m.self_reduce_ll16(x, y, pk.ptr, out, flags, err)
        ho.copy_(out, non_blocking=True)

    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / reps
    return {"value": round(S / t / 1e9, 2), "unit": "GB/s", "ms_per_step": round(t * 1e3, 3),
            "note": "S / (H2D 2S + pack+sum+unpack + D2H S) with host-pinned buffers (PCIe-inclusive)"}


def bench_single(args):
    import mscclpp_amd as m

    hp = None if args.no_cpu_baseline else host_proxy_baseline()
    S = args.bytes
    count = S // 2
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.rand(count, generator=g).to(torch.float16).to(dev)
    y = torch.rand(count, generator=g).to(torch.float16).to(dev)
    out = torch.empty_like(x)
    pk = m.DeviceBuffer(2 * S)
    flags = torch.ones(m.FLAG_SLOTS, dtype=torch.int32, device=dev)
    err = torch.zeros(16, dtype=torch.int32, device=dev)

    def step():
        m.self_reduce_ll16(x, y, pk.ptr, out, flags, err)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # timed region: exactly K steps, synchronize on both sides.  The kernel's average launch duration
    # comes from a HIP event pair on the launch stream (torch's current stream, which
    # self_reduce_ll16 launches on) bracketing the same K back-to-back launches.
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        step()
    ev1.record()
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / args.steps
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    assert int(err[0].item()) == 0, "device error word set"
    # correctness spot check of the last step
    ref = (x.float() + y.float()).clamp(-65504, 65504).half()
    assert torch.equal(out, ref), "self-reduce mismatch"
    achieved = 7 * S / (kern_ms * 1e-3) / 1e9
    res = {
        "metric": "device-resident AllReduce algbw GB/s fp16 at 1/2/4/8 MI355X; % xGMI roofline",
        "value": round(S / t / 1e9, 2),
        "unit": "GB/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(t * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f16",
        "data": "synthetic",
        "config": {"workload": "ll16_self_reduce_fp16_48MiB (BASELINE configs[1]: pack+sum+unpack, 1 GPU)",
                   "bytes": S, "parallelism": "single-gpu"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": committed_traffic(S),
                     "kernel": "selfReduceLL16LdsKernel", "kernel_us": round(kern_ms * 1e3, 2),
                     "algorithmic_bytes_per_launch": 7 * S},
    }
    if args.no_extras:  # profiling runs: only the headline launches, so per-kernel stats are of one size
        pk.free()
        return res
    res["staged_pcie_inclusive"] = staged_rate(m, S, x, y, out, pk, flags, err)
    # BASELINE configs[1] sweep, 64 KiB .. 48 MiB: per-launch time with 20 launches captured in one
    # HIP graph (device time, not host launch rate)
    sweep = {}
    for sz in (64 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20, 48 << 20):
        if sz > S:
            break
        xs, ys, os_ = x[: sz // 2], y[: sz // 2], out[: sz // 2]
        us = graph_time_per_call(lambda: m.self_reduce_ll16(xs, ys, pk.ptr, os_, flags, err)) * 1e6
        sweep[f"{sz >> 10}KiB"] = {"kernel_us": round(us, 2), "algbw_GBs": round(sz / us / 1e3, 1),
                                   "hbm_7S_TBs": round(7 * sz / us / 1e6, 3)}
    res["sweep"] = sweep
    if not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline_self_reduce(S, args.cpu_seconds)
        res["host_proxy_baseline"] = hp
    pk.free()
    return res


def _time_calls(fn, reps):
    """Mean per-call time (s) of `reps` back-to-back calls, synchronised on both sides."""
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def progress(msg):
    """Stage markers on stderr (rank 0): a long multi-GPU run keeps writing, and a stall names its stage."""
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def bench_multi(args):
    import torch.distributed as dist

    import mscclpp_amd as m

    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    ndev = torch.cuda.device_count()
    if ndev < world:  # rehearsal on a smaller box: ranks share devices (never the case on the 8-GPU node)
        local = local % ndev
    torch.cuda.set_device(local)
    # a rank that stalls must turn into an error (caught per extras section) well before the driver's
    # limit, so the JSON line is still printed: bounded bootstrap and gloo timeouts
    os.environ.setdefault("MSCCLPP_AMD_BOOTSTRAP_TIMEOUT_S", "180")
    import datetime

    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=300))
    comm = m.Communicator.from_torch_dist()
    n = world
    S = args.bytes
    count = S // 2
    dev = torch.device("cuda", local)
    g = torch.Generator(device="cpu").manual_seed(rank)
    x = torch.rand(count, generator=g).to(torch.float16).to(dev)
    out = torch.empty_like(x)

    def tmax(v):
        t = torch.tensor([v], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t[0])

    # ---- pick the algorithm and launch shape (untimed; every rank tries the same candidates in the
    # same order).  Large buckets: the scratch-based all-pairs RS+AG (fullmesh, puts) and the
    # zero-copy RS+AG (reads peers' inputs, writes peers' outputs) -- which one drives xGMI better
    # is measured here, on the node, not assumed.
    sel = {1: "packet", 2: "allpair", 3: "fullmesh", 4: "rsag", 5: "rsag_zc"}[m.lib().mscclppAmdSelectAlgo(n, S, 0)]
    algos = [args.algo] if args.algo else ([sel, "rsag_zc", "rsag_pipeline"] if sel == "fullmesh" else [sel])
    cands = []
    shared = ndev < world  # rehearsal: ranks share a device, so every rank's grid must fit on it at once
    for a in algos:
        if a in ("fullmesh", "rsag", "rsag_zc"):
            cands += [(a, nb_, nt_) for nb_, nt_ in ((64, 512), (128, 512), (256, 512), (128, 256), (256, 256))
                      if not shared or nb_ * world <= 256]
        elif a == "rsag_pipeline":  # nblocks = reduce workgroups; the launch is 2x that
            cands += [(a, nb_, nt_) for nb_, nt_ in ((32, 512), (64, 512), (128, 512), (64, 256))
                      if not shared or 2 * nb_ * world <= 256]
        else:
            cands.append((a, 0, 0))
    tune = {}
    progress(f"tuning {len(cands)} candidates")
    for a, nb, nt in cands:
        try:
            for _ in range(2):
                comm.all_reduce(x, out, algo=a, nblocks=nb, nthreads=nt)
            tune[(a, nb, nt)] = tmax(_time_calls(lambda: comm.all_reduce(x, out, algo=a, nblocks=nb, nthreads=nt), 5))
        except Exception as e:  # a rejected shape is simply skipped
            tune[(a, nb, nt)] = float("inf")
            if rank == 0:
                print(f"tune {a} {nb}x{nt}: {e}", file=sys.stderr)
    if tmax(float(comm.device_error())) != 0:  # a spin timed out somewhere: say so instead of hanging on
        print("bench: device error after tuning; results below are suspect", file=sys.stderr)
    algo, nb, nt = min(tune, key=tune.get)

    def step():
        comm.all_reduce(x, out, algo=algo, nblocks=nb, nthreads=nt)

    progress(f"selected {algo} {nb}x{nt}; warmup + timed region")
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # ---- timed region: exactly K steps, barrier + synchronize on both sides, max over ranks; the
    # kernel duration from an event pair on the launch stream around the same K launches
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        step()
    ev1.record()
    torch.cuda.synchronize()
    t_local = (time.perf_counter() - t0) / args.steps
    dist.barrier()
    t = tmax(t_local)
    kern_ms = tmax(ev0.elapsed_time(ev1) / args.steps)
    errc = comm.device_error()
    # correctness of the timed call: fp32 gloo reference of the same inputs (tolerance of
    # python/mscclpp_benchmark/correctness.py:257-258)
    ref = x.float().cpu()
    dist.all_reduce(ref)
    ok = bool(torch.allclose(out.float().cpu(), ref, rtol=1e-2, atol=5e-4 * n)) and errc == 0
    algbw = S / t / 1e9
    ceiling = n * XGMI_LINK_GBS / 2  # all-pairs algbw ceiling
    # HBM bytes one rank's AllReduce moves.  fullmesh/rsag: reads S input + (n-1)/n S scratch;
    # writes S/n own output + (n-1)/n S incoming scratch + (n-1)/n S incoming output.  rsag_zc: reads
    # S of input (own slice locally, the rest by the peers), writes S of output (own slice locally,
    # the rest by the peers).  LL paths: priced like fullmesh (their packets double the bytes).
    # rsag_pipeline: reads S input + 2(n-1)/n S scratch (RS and AG regions), writes S output +
    # 2(n-1)/n S incoming scratch
    hbm = (2 * S if algo == "rsag_zc" else 2 * S * (1 + 2 * (n - 1) / n) if algo == "rsag_pipeline"
           else S * (1 + 3 * (n - 1) / n + 1 / n))
    res = {
        "metric": "device-resident AllReduce algbw GB/s fp16 at 1/2/4/8 MI355X; % xGMI roofline",
        "value": round(algbw, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(t * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f16",
        "data": "synthetic",
        "config": {"workload": f"allreduce_fp16_{S >> 20}MiB (BASELINE configs[2]: 2048x12288 fp16 bucket per rank)",
                   "bytes": S, "parallelism": f"allreduce{world}", "algo": algo, "nblocks": nb, "nthreads": nt},
        "busbw": round(algbw * 2 * (n - 1) / n, 2),
        "xgmi": {"allpairs_algbw_ceiling": round(ceiling, 1), "frac": round(algbw / ceiling, 4),
                 "link_GBs_assumed": XGMI_LINK_GBS, "wire_bytes_per_rank": int(2 * (n - 1) * S / n)},
        "roofline": {"bound": "hbm", "achieved": round(hbm / (kern_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "traffic": None, "kernel": {"rsag_zc": "allreduceZeroCopyKernel", "rsag_pipeline": "allreduceRsAgPipelineKernel"}.get(algo, f"allreduceBulkKernel ({algo})"),
                     "kernel_us": round(kern_ms * 1e3, 2), "algorithmic_bytes_per_launch": int(hbm)},
        "tune_ms": {f"{k[0]}:{k[1]}x{k[2]}": round(v * 1e3, 4) for k, v in tune.items()},
        "correct": ok,
    }
    res["roofline"]["frac"] = round(res["roofline"]["achieved"] / HBM_PEAK_GBS, 4)
    if not args.no_extras:
        progress("xGMI probe")
        try:
            probe = xgmi_probe(comm, n, dev, tmax, dist.barrier)
            res["xgmi"]["measured"] = probe
            res["xgmi"]["frac_of_measured_ceiling"] = round(algbw / probe["allpairs_algbw_ceiling_measured"], 4)
        except Exception as e:  # recorded, never fatal for the headline line
            res["xgmi"]["measured_error"] = str(e)[-300:]
        res["extras"] = bench_extras(args, comm, n, dev, tmax, dist.barrier)
    # cpu_baseline is an N=1 field (the oracle timed on rank 0 at N=1 only); at N>1 the reference's
    # host-proxy path is reported by the mscclpp-test k1 row in extras
    comm.destroy()
    dist.barrier()
    dist.destroy_process_group()
    return res if rank == 0 else None


def xgmi_probe(comm, n, dev, tmax, barrier, S=64 << 20):
    """Raw xGMI ceilings measured on the node (calibrate B_link with a raw put
    microbenchmark): the streaming copy kernel (mscclppAmdCopy, 16-byte loads/stores over all CUs)
    with one side in IPC-mapped peer memory.  ring_put: every rank writes S into the next rank (each
    link carries one direction); ring_get: every rank reads S from the previous rank; allpairs_put:
    every rank writes S/(n-1) into each peer at once (one stream per peer).  Max over ranks."""
    import mscclpp_amd as m

    L = m.lib()
    rank = comm.rank
    src = torch.full((S,), rank & 0xFF, dtype=torch.uint8, device=dev)
    dst = torch.empty(S, dtype=torch.uint8, device=dev)
    pdst = comm.register_buffer(dst)
    psrc = comm.register_buffer(src)
    nxt, prv = (rank + 1) % n, (rank - 1) % n
    vp = ctypes.c_void_p

    def timed(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return tmax((time.perf_counter() - t0) / reps)

    sp = m.stream_ptr()
    t_put = timed(lambda: L.mscclppAmdCopy(vp(src.data_ptr()), vp(pdst[nxt]), S, 1024, sp))
    t_get = timed(lambda: L.mscclppAmdCopy(vp(psrc[prv]), vp(dst.data_ptr()), S, 1024, sp))
    chunk = (S // (n - 1)) // 16 * 16
    peers = [q for q in range(n) if q != rank]
    streams = [torch.cuda.Stream(device=dev) for _ in peers]
    nb = max(64, 1024 // (n - 1))

    def allpairs():
        for st in streams:
            st.wait_stream(torch.cuda.current_stream())
        for i, q in enumerate(peers):
            slot = (rank - q - 1) % n  # distinct destination region per source
            L.mscclppAmdCopy(vp(src.data_ptr() + i * chunk), vp(pdst[q] + slot * chunk), chunk, nb, m.stream_ptr(streams[i]))
        for st in streams:
            torch.cuda.current_stream().wait_stream(st)

    t_ap = timed(allpairs)
    barrier()
    out = {"bytes": S, "ring_put_GBs": round(S / t_put / 1e9, 1), "ring_get_GBs": round(S / t_get / 1e9, 1),
           "allpairs_put_out_GBs": round((n - 1) * chunk / t_ap / 1e9, 1)}
    # all-pairs AllReduce moves 2(n-1)/n * S out of every rank: its algbw ceiling at the measured rate
    out["allpairs_algbw_ceiling_measured"] = round(out["allpairs_put_out_GBs"] * n / (2 * (n - 1)), 1)
    return out


def graph_time_per_call(fn, calls=20, replays=10, sync=None):
    """Per-call time with `calls` calls captured in one HIP graph (mscclpp-test common.cc:202-227).
    `sync` (a host barrier across ranks) lines the ranks up before the timed replays, so the first
    replay does not absorb another rank's late start."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(calls):
            fn()
    g.replay()
    torch.cuda.synchronize()
    if sync is not None:
        sync()
    return _time_calls(g.replay, replays) / calls


def bench_extras(args, comm, n, dev, tmax, barrier):
    """BASELINE configs[3] (LL latency sweep, fp16 1 KiB..1 MiB) and configs[4] (fp32 1 GiB
    RS+AG in ring order), timed the same way; failures are recorded, not raised."""
    extras = {}
    progress("extras: LL latency sweep")
    try:
        lat = {}
        for kb in (1, 4, 16, 64, 256, 1024):
            cnt = kb * 512
            xs = torch.rand(cnt, device=dev).half()
            os_ = torch.empty_like(xs)
            for _ in range(5):
                comm.all_reduce(xs, os_)
            torch.cuda.synchronize()
            barrier()
            lat[f"{kb}KiB"] = round(tmax(_time_calls(lambda: comm.all_reduce(xs, os_), 50)) * 1e6, 2)
        extras["ll_latency_us"] = lat
    except Exception as e:
        extras["ll_latency_error"] = str(e)
    try:
        glat = {}
        # the first graph a process times runs slow (a one-time cost, tools/ll_small_probe.py:
        # 32 us for the first size, 3.3 us for the same size measured again) -- discard one
        xw = torch.rand(512, device=dev).half()
        graph_time_per_call(lambda: comm.all_reduce(xw, torch.empty_like(xw)), sync=barrier)
        for kb in (1, 4, 16, 64, 256, 1024):
            cnt = kb * 512
            xs = torch.rand(cnt, device=dev).half()
            os_ = torch.empty_like(xs)
            glat[f"{kb}KiB"] = round(tmax(graph_time_per_call(lambda: comm.all_reduce(xs, os_), sync=barrier)) * 1e6, 2)
        extras["ll_latency_graph_us"] = glat
    except Exception as e:
        extras["ll_latency_error"] = str(e)
    progress("extras: fp32 1 GiB rsag")
    try:
        S = 1 << 30
        xs = torch.rand(S // 4, device=dev)
        os_ = torch.empty_like(xs)
        for _ in range(2):
            comm.all_reduce(xs, os_, algo="rsag")
        t = tmax(_time_calls(lambda: comm.all_reduce(xs, os_, algo="rsag"), 5))
        extras["fp32_1GiB_rsag"] = {"ms": round(t * 1e3, 3), "algbw_GBs": round(S / t / 1e9, 2),
                                    "busbw_GBs": round(S / t / 1e9 * 2 * (n - 1) / n, 2)}
        del xs, os_
    except Exception as e:
        extras["fp32_1GiB_rsag_error"] = str(e)
    progress("extras: mscclpp-test kernels")
    try:
        # the mscclpp-test kernels on the sizes the reference publishes (BASELINE.md §1,
        # test/deploy/perf_ndmv4.jsonl / perf_ndmv5.jsonl), timed like common.cc:202-227
        # (20 calls in one graph, 15 launches), int32 data = rank
        mt = {}
        for k, kb, pub in (("k6", 24, "A100 7.24 us / H100 6.18 us"), ("k6", 48, "A100 7.91 us / H100 6.62 us"),
                           ("k6", 72, "A100 8.28 us / H100 6.91 us"), ("k7", 48, None),
                           ("k5", 48 << 10, "A100 397.79 us, 126.52 GB/s")):
            cnt = kb * 256
            if (kb << 10) % (16 * n):
                continue
            xs = torch.full((cnt,), comm.rank, dtype=torch.int32, device=dev)
            os_ = xs if k == "k5" else torch.empty_like(xs)
            us = tmax(graph_time_per_call(lambda: comm.all_reduce(xs, os_, algo=k), calls=20, replays=15,
                                          sync=barrier)) * 1e6
            row = {"us": round(us, 2), "algbw_GBs": round((kb << 10) / us / 1e3, 2)}
            if pub:
                row["reference_published"] = pub
            mt[f"{k}_{kb}KiB" if kb < 1024 else f"{k}_{kb >> 10}MiB"] = row
            del xs, os_
        # allreduce1: the int32 ring whose bytes move through PortChannels and the host proxy
        # (perf_ndmv4.jsonl:4: 1 GiB, 7701.98 us, 139.41 GB/s on 8 x A100)
        barrier()
        comm.deregister_all()
        us, ok, _ = comm.proxy_ring_all_reduce((1 << 30) // 4, iters=3, graph_launches=2)
        us = tmax(us)
        mt["k1_1GiB"] = {"us": round(us, 1), "algbw_GBs": round((1 << 30) / us / 1e3, 2), "correct": ok,
                         "reference_published": "A100 7701.98 us, 139.41 GB/s"}
        extras["mscclpp_test"] = mt
    except Exception as e:
        extras["mscclpp_test_error"] = str(e)
    extras["device_error"] = comm.device_error()
    return extras


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        res = bench_multi(args)
    else:
        res = bench_single(args)
    if res is not None:
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
