"""mscclpp_amd benchmark (driver contract: one JSON line on rank 0).

N = 1  -> BASELINE.json configs[1]: the 1-GPU LL16 pack + sum + unpack self-reduce, fp16, 48 MiB,
          device-resident (the HBM-roofline check of the LL hot path).
N > 1  -> BASELINE.json configs[2]: ncclAllReduce of a 48 MiB fp16 bucket (2048 x 12288, the
          README's GPT-3 TP bucket) per rank, one process per GPU, one-sided puts over xGMI
          through libmscclpp_amd.so (no RCCL underneath).  Launched either by torch.distributed.run
          (RANK / WORLD_SIZE set) or by this script itself: `python bench.py --gpus N` with no
          WORLD_SIZE spawns N rank processes from a parent that never touches the GPU.

value = algbw = S / t (GB/s): S = bucket bytes per rank, t = max over ranks of the time per step
inside the timed region (barrier + synchronize on both sides).  Inputs are resident in HBM before
the timed region starts.  The roofline object prices the dominant kernel with its live HIP-event
duration.  Test infrastructure under oracle/ (liboracle.so through tests/oracle_lib.py) is used
only as a checker outside the timed region: cpu_baseline (N = 1) and the bit-exact correctness
check of the N > 1 results.
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
    p.add_argument("--gpus", type=int, default=None,
                   help="ranks (one GPU each); default: WORLD_SIZE if set, else 1.  N > 1 without WORLD_SIZE "
                        "spawns the N rank processes")
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--bytes", type=int, default=48 << 20)
    p.add_argument("--algo", default=None,
                   help="force an AllReduce algorithm (N>1): packet|allpair|fullmesh|rsag|rsag_zc|rsag_pipeline")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-extras", action="store_true", help="N>1: skip the LL latency sweep and the fp32 1 GiB run")
    p.add_argument("--no-check", action="store_true", help="N>1: skip the per-candidate bit-exact checks")
    p.add_argument("--same-input", action="store_true", help="N>1 diagnostic: every step on the seq-1 input")
    p.add_argument("--dry-run", action="store_true",
                   help="launcher self-test: every rank checks its environment, rank 0 prints the rank layout")
    p.add_argument("--rank-timeout", type=float, default=1500.0, help="launcher: seconds before hung ranks are killed")
    return p.parse_args()


def cpu_threads():
    """Threads for the all-core CPU figures: the CPUs this process may use, capped by OMP_NUM_THREADS
    where the pool sets it (16 per GPU on the GPU boxes, whose nproc shows the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return max(1, min(n, int(omp))) if omp.isdigit() and int(omp) > 0 else n


def _parallel_rate(work, threads, budget_s, max_iters):
    """Run work(t) for t in range(threads) on a thread pool (the oracle's ctypes calls release the
    GIL), repeatedly until budget_s; returns (iterations, seconds).  One untimed warm pass first."""
    import concurrent.futures as cf

    with cf.ThreadPoolExecutor(threads) as ex:
        list(ex.map(work, range(threads)))
        iters, t0 = 0, time.perf_counter()
        while True:
            list(ex.map(work, range(threads)))
            iters += 1
            el = time.perf_counter() - t0
            if el >= budget_s or iters >= max_iters:
                return iters, el


def _sum_parts(n_src, nbytes, threads):
    """The inputs, output and per-thread slices of cpu_baseline_sum."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O

    nw = nbytes // 4
    ins = [O.lcg(O.F16, nbytes // 2, r, 0).view(np.uint32) for r in range(n_src)]
    out = np.empty(nw, np.uint32)
    parts = []
    for t in range(threads):
        a, b = nw * t // threads, nw * (t + 1) // threads
        parts.append(((ctypes.c_void_p * n_src)(*[x.ctypes.data + 4 * a for x in ins]), b - a,
                      ctypes.c_void_p(out.ctypes.data + 4 * a)))

    def work(t):
        srcs, words, dst = parts[t]
        if words:
            O.L().oracle_reduce_seq(O.F16, O.SUM, n_src, srcs, words, dst)

    return ins, out, work


def _threaded_sum_for_test(n_src, nbytes, threads):
    ins, out, work = _sum_parts(n_src, nbytes, threads)
    for t in range(threads):
        work(t)
    return out


def cpu_baseline_sum(n_src, nbytes, budget_s, threads=None):
    """SURVEY §8(d)'s CPU context figure: the oracle's fp16 n-way sum (own, then ascending -- the
    fullmesh order of rank 0, oracle_reduce_seq) of n LCG buckets of `nbytes`, the bucket split over
    `threads` threads; GB/s = result bytes (one bucket per AllReduce) per second, as `value`."""
    threads = threads or cpu_threads()
    ins, out, work = _sum_parts(n_src, nbytes, threads)
    iters, el = _parallel_rate(work, threads, budget_s, 1000)
    return {"value": round(nbytes * iters / el / 1e9, 3), "unit": "GB/s", "cores": threads, "kind": "port",
            "nproc": os.cpu_count(),
            "sample": f"{iters} x oracle fp16 {n_src}-way sum (own then ascending) of {n_src} x {nbytes >> 20} MiB "
                      f"LCG buckets, split over {threads} threads, in {el:.1f} s"}


def cpu_baseline_self_reduce(nbytes, budget_s, threads=1):
    """The N=1 workload itself on the CPU: the oracle's pack + sum + unpack (oracle_self_reduce) of
    the same 48 MiB fp16 bucket, split over `threads` threads (LL16 packets pair words: even slices)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O

    nw = nbytes // 4
    x = O.lcg(O.F16, nbytes // 2, 0, 0).view(np.uint32)
    y = O.lcg(O.F16, nbytes // 2, 1, 0).view(np.uint32)
    pk = np.empty(2 * nw, np.uint32)
    out = np.empty(nw, np.uint32)
    L = O.L()
    cut = [nw * t // threads // 2 * 2 for t in range(threads)] + [nw]

    def work(t):
        a, b = cut[t], cut[t + 1]
        if b > a:
            L.oracle_self_reduce(O.F16, O.SUM, ctypes.c_void_p(x.ctypes.data + 4 * a),
                                 ctypes.c_void_p(y.ctypes.data + 4 * a), b - a, 1,
                                 ctypes.c_void_p(pk.ctypes.data + 8 * a), ctypes.c_void_p(out.ctypes.data + 4 * a))

    iters, el = _parallel_rate(work, threads, budget_s, 200)
    return {"value": round(nbytes * iters / el / 1e9, 3), "unit": "GB/s", "cores": threads, "kind": "port",
            "sample": f"{iters} x oracle_self_reduce fp16 {nbytes >> 20} MiB (pack + sum + unpack, scalar C) "
                      f"over {threads} thread(s) in {el:.1f} s"}


def committed_traffic(S):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/<tag>_self_reduce_pmc.json:
    2*FETCH_SIZE + WRITE_SIZE, the gfx950 correction of MI355X_MICROARCH.md §HBM), or None."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_self_reduce_pmc.json")))
    if not files or S != 48 << 20:
        return None
    d = json.load(open(files[-1]))
    return d.get("hbm_bytes_per_launch_corrected")


def committed_multirank_pmc(kernel):
    """read / write byte ratios of `kernel` from profiles/*_multirank_pmc.json (tools/pmc_multirank.sh), or None."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_multirank_pmc.json")))
    if not files:
        return None
    ks = json.load(open(files[-1])).get("kernels", {})
    name = {"allreduceZeroCopyKernel": "allreduceZeroCopyKernel<0, 0, 8>"}.get(
        kernel, "allreduceBulkKernel<0, 0, 8, 0, 0>" if kernel.startswith("allreduceBulkKernel") else None)
    k = ks.get(name) if name else None
    return None if k is None else {"read_ratio": k["read_ratio"], "write_ratio": k["write_ratio"],
                                   "source": os.path.basename(files[-1])}


def host_proxy_baseline(n=2, timeout=240):
    """The reference's host-proxy path (test/allgather_test_host_offloading.cu, 4 KiB) on n ranks --
    spawned before this process touches the GPU.  N=1: BASELINE config 1 (2 ranks, loopback); N>1:
    the same loop at the job's world size, one rank per GPU (2 cores per rank).  Its
    processes are killed when they have not all answered within `timeout` seconds."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    try:
        import host_proxy_baseline as H

        return H.run(n, 4096, timeout=timeout)
    except Exception as e:  # recorded, never fatal for the headline line
        return {"error": str(e)[-400:]}


def pingpong_extras(hp):
    """The N=1 line's extras: the reference's MemoryChannel packet ping-pong latency
    (memory_channel_tests.cu:98-107), measured by the two host-proxy ranks (tools/host_proxy_baseline.py),
    labelled by where those ranks ran: one shared GPU, or two GPUs one xGMI hop apart."""
    hp = hp or {}
    pp = hp.get("pingpong") or {}
    devs = hp.get("devices") or []
    if len(devs) == 1:
        where = "two processes on ONE GPU through IPC-mapped packet buffers: a shared-device figure, not an xGMI latency"
    elif len(devs) == 2:
        where = f"two processes on GPUs {devs} through IPC-mapped peer packet buffers: one xGMI hop"
    else:
        where = "not measured: " + str(hp.get("error", "no host-proxy ranks"))[-200:]
    return {"ll16_pingpong_us": (pp.get("ll16") or {}).get("us_per_iter"),
            "ll8_pingpong_us": (pp.get("ll8") or {}).get("us_per_iter"),
            "pingpong_correct": hp.get("pingpong_correct"),
            "pingpong_devices": devs,
            "pingpong_note": "us per one-way hand-off of 1024 ints (100k timed iterations, 1 workgroup per rank), "
                             + where}


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
    res = {"value": round(S / t / 1e9, 2), "unit": "GB/s", "ms_per_step": round(t * 1e3, 3),
           "note": "S / (H2D 2S + pack+sum+unpack + D2H S) with host-pinned buffers (PCIe-inclusive)"}
    # zero-copy staging: the kernel reads X, Y straight out of the pinned host buffers and writes O
    # straight back over PCIe (the packets stay in HBM), so both directions of the link run at once
    # with no copy-engine hops (tools/staging_probe.py)
    def zero_copy():
        m.self_reduce_ll16(hx, hy, pk.ptr, ho, flags, err)

    zero_copy()
    torch.cuda.synchronize()
    ho_ref = ho.clone()
    t0 = time.perf_counter()
    for _ in range(reps):
        zero_copy()
    torch.cuda.synchronize()
    tz = (time.perf_counter() - t0) / reps
    step()  # the copy path's result for the same inputs
    torch.cuda.synchronize()
    res["zero_copy"] = {"value": round(S / tz / 1e9, 2), "ms_per_step": round(tz * 1e3, 3),
                        "correct": bool(torch.equal(ho_ref, ho)),
                        "note": "the kernel reads X, Y from and writes O to the host-pinned buffers directly (PCIe both ways at once)"}
    return res


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
        "scaling_note": SCALING_NOTE,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": committed_traffic(S),
                     "kernel": "selfReduceLL16LdsKernel", "kernel_us": round(kern_ms * 1e3, 2),
                     "algorithmic_bytes_per_launch": 7 * S,
                     # BASELINE.md §3 row 2's secondary figure: the HBM reads alone (Y, P, X = 4*S)
                     "read_only": {"bytes_per_launch": 4 * S,
                                   "achieved": round(4 * S / (kern_ms * 1e-3) / 1e9, 1),
                                   "frac": round(4 * S / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}},
    }
    if args.no_extras:  # profiling runs: only the headline launches, so per-kernel stats are of one size
        pk.free()
        return res
    # the same run's ceilings beside the headline: a streaming copy of the
    # bucket (read S + write S), and the kernel from a cold Infinity Cache (a 512 MiB write between
    # launches evicts the 240 MiB working set that back-to-back launches find in the 256 MiB MALL)
    res["roofline"].update(same_run_ceilings(m, S, x, y, pk, out, flags, err, kern_ms))
    res["staged_pcie_inclusive"] = staged_rate(m, S, x, y, out, pk, flags, err)
    # BASELINE configs[1] sweep, 64 KiB .. 48 MiB in x2 steps: per-launch time with 20 launches
    # captured in one HIP graph (device time, not host launch rate)
    sweep = {}
    for sz in [(64 << 10) << k for k in range(10)] + [48 << 20]:
        if sz > S:
            break
        xs, ys, os_ = x[: sz // 2], y[: sz // 2], out[: sz // 2]
        us = graph_time_per_call(lambda: m.self_reduce_ll16(xs, ys, pk.ptr, os_, flags, err)) * 1e6
        sweep[f"{sz >> 10}KiB"] = {"kernel_us": round(us, 2), "algbw_GBs": round(sz / us / 1e3, 1),
                                   "hbm_7S_TBs": round(7 * sz / us / 1e6, 3)}
    res["sweep"] = sweep
    if not args.no_cpu_baseline:
        # the oracle's fp16 8-way sum on the box's cores; beside it the N=1 workload
        # itself (pack + sum + unpack) on one core and on all of them, and the host-proxy path
        res["cpu_baseline"] = cpu_baseline_sum(8, S, args.cpu_seconds)
        res["cpu_baseline_self_reduce"] = {"1_thread": cpu_baseline_self_reduce(S, args.cpu_seconds / 2, 1),
                                           "all_threads": cpu_baseline_self_reduce(S, args.cpu_seconds / 2,
                                                                                   cpu_threads())}
        res["host_proxy_baseline"] = hp
        # the reference's MemoryChannel packet ping-pong latency (memory_channel_tests.cu:98-107), from
        # the same two host-proxy ranks: on a 1-GPU box both ranks share the GPU
        res["extras"] = pingpong_extras(hp)
    pk.free()
    return res


def same_run_ceilings(m, S, x, y, pk, out, flags, err, kern_ms, reps=20):
    """Copy ceiling and cold-cache time of the headline kernel, measured in this run."""
    L = m.lib()
    vp = ctypes.c_void_p
    dst = torch.empty_like(x)

    def copy():
        m.check(L.mscclppAmdCopy(vp(x.data_ptr()), vp(dst.data_ptr()), S, 0, m.stream_ptr()), "copy")

    copy()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        copy()
    b.record()
    torch.cuda.synchronize()
    copy_us = a.elapsed_time(b) * 1e3 / reps
    copy_gbs = 2 * S / (copy_us * 1e-6) / 1e9

    def stream():  # the self-reduce's exact 7*S access mix with no hand-off (mscclppAmdSelfReduceStream)
        m.check(L.mscclppAmdSelfReduceStream(vp(x.data_ptr()), vp(y.data_ptr()), vp(pk.ptr), vp(dst.data_ptr()), S,
                                             m.stream_ptr()), "stream mix")

    stream()
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        stream()
    b.record()
    torch.cuda.synchronize()
    mix_us = a.elapsed_time(b) * 1e3 / reps
    mix_gbs = 7 * S / (mix_us * 1e-6) / 1e9
    # an independent ceiling of the same 4:3 read:write mix: a generic grid-stride kernel with none
    # of the self-reduce's layout, grid or rounds (mscclppAmdMixStream), separate write buffers
    pout = torch.empty(2 * S, dtype=torch.uint8, device=x.device)

    def generic():
        m.check(L.mscclppAmdMixStream(vp(x.data_ptr()), vp(y.data_ptr()), vp(pk.ptr), vp(pout.data_ptr()),
                                      vp(dst.data_ptr()), S, 0, m.stream_ptr()), "generic mix")

    generic()
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        generic()
    b.record()
    torch.cuda.synchronize()
    gen_us = a.elapsed_time(b) * 1e3 / reps
    gen_gbs = 7 * S / (gen_us * 1e-6) / 1e9
    del pout
    scrub = torch.empty(512 << 20, dtype=torch.uint8, device=x.device)

    def one_pair(cold):
        if cold:
            scrub.fill_(1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        m.self_reduce_ll16(x, y, pk.ptr, out, flags, err)
        e1.record()
        return e0, e1

    res = {}
    for name, cold in (("warm_pair", False), ("cold", True)):
        evs = [one_pair(cold) for _ in range(reps)]
        torch.cuda.synchronize()
        res[name] = float(np.median([e0.elapsed_time(e1) * 1e3 for e0, e1 in evs]))
    del scrub, dst
    seven = 7 * S
    return {"copy_ceiling_GBs": round(copy_gbs, 1), "copy_ceiling_frac": round(copy_gbs / HBM_PEAK_GBS, 4),
            "copy_us": round(copy_us, 2),
            "frac_of_copy_ceiling": round(seven / (kern_ms * 1e-3) / 1e9 / copy_gbs, 4),
            "mix_ceiling_GBs": round(mix_gbs, 1), "mix_ceiling_frac": round(mix_gbs / HBM_PEAK_GBS, 4),
            "mix_us": round(mix_us, 2), "frac_of_mix_ceiling": round(seven / (kern_ms * 1e-3) / 1e9 / mix_gbs, 4),
            "mix_note": "mix: the kernel's own 7*S accesses on the same buffers, grid and rounds with no flags, "
                        "polls or LDS (mscclppAmdSelfReduceStream)",
            "generic_mix_ceiling_GBs": round(gen_gbs, 1), "generic_mix_us": round(gen_us, 2),
            "frac_of_generic_mix_ceiling": round(seven / (kern_ms * 1e-3) / 1e9 / gen_gbs, 4),
            "generic_mix_note": "an independent ceiling of the 4:3 read:write mix: a grid-stride kernel over 16-byte "
                                "units, 2048 x 256 lanes, nt accesses, separate write buffers (mscclppAmdMixStream)",
            "cold": {"kernel_us": round(res["cold"], 2),
                     "achieved": round(seven / (res["cold"] * 1e-6) / 1e9, 1),
                     "frac": round(seven / (res["cold"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                     "warm_same_method_us": round(res["warm_pair"], 2),
                     "method": "median of 20 launches, one event pair each; cold: a 512 MiB fill before each launch"},
            "note": "frac is the warm back-to-back replay (the 240 MiB working set fits the 256 MiB Infinity Cache); "
                    "cold and the same run's streaming-copy ceiling beside it"}


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


SELECT_NAMES = {1: "packet", 2: "allpair", 3: "fullmesh", 4: "rsag", 5: "rsag_zc", 6: "rsag_pipeline"}
FULL_NAMES = {"packet": "default_allreduce_packet", "allpair": "default_allreduce_allpair_packet",
              "fullmesh": "default_allreduce_fullmesh", "rsag": "default_allreduce_rsag",
              "rsag_zc": "default_allreduce_rsag_zero_copy", "rsag_pipeline": "default_allreduce_rsag_pipeline"}

SCALING_NOTE = ("n_gpus=1 measures BASELINE configs[1] (the 1-GPU LL16 pack+sum+unpack of a 48 MiB fp16 bucket, "
                "S / kernel-step time); n_gpus>1 measures configs[2] (AllReduce algbw S / t of a 48 MiB fp16 bucket per "
                "rank over xGMI).  Different workloads: the 1 -> N ratio is not the scaling efficiency of one workload.")


def lcg_tensor(count, rank, seq, dtype, dev):
    """test/torch/correctness_test.py:19-22, 44-56 on the device: v_i = ((((i + rank + seq) & M) * 1664525 +
    1013904223) & M) % 4096 / 4096, cast RNE (the oracle's oracle_lcg_fill generates the same values on the CPU)."""
    i = torch.arange(count, dtype=torch.int64, device=dev)
    s = (i + rank + seq) & 0xFFFFFFFF
    s = (s * 1664525 + 1013904223) & 0xFFFFFFFF
    return ((s % 4096).to(torch.float32) / 4096.0).to(dtype)


RING_CHUNK = 1 << 25  # elements per generator call of the fp32 ring check (bounds its int64 temporaries)


def ring_bits(i, rank, seq):
    """Order-sensitive fp32 inputs of configs[4] (the 1 GiB ring-order RS+AG): a 32-bit hash of
    (element i, rank, seq) laid out as IEEE bits -- random sign, exponent 2^0 .. 2^-7, full 23-bit
    mantissa -- so that a sum of n ranks' values rounds differently in different orders (the LCG of
    lcg_tensor makes multiples of 1/4096, whose fp32 sums are exact in ANY order and would let a
    wrong order pass).  `i` is an int64 numpy array or torch tensor; every product stays below 2^63.
    Returns the bits as signed int64 (view them as int32 -> float32)."""
    M = 0xFFFFFFFF
    s = (i + rank * 0x9E3779B1 + seq * 0x7F4A7C15) & M
    s = (s * 1664525 + 1013904223) & M
    s = s ^ (s >> 15)
    s = (s * 0x2C1B3C6D) & M
    s = s ^ (s >> 13)
    sign = (s >> 31) & 1
    bits = (sign << 31) | ((127 - ((s >> 23) & 7)) << 23) | (s & 0x7FFFFF)
    return bits - (sign << 32)


def ring_tensor(start, count, rank, seq, dev):
    """ring_bits of elements [start, start + count) as a float32 tensor on `dev`."""
    out = torch.empty(count, dtype=torch.float32, device=dev)
    for a in range(0, count, RING_CHUNK):
        b = min(count, a + RING_CHUNK)
        i = torch.arange(start + a, start + b, dtype=torch.int64, device=dev)
        out[a:b] = ring_bits(i, rank, seq).to(torch.int32).view(torch.float32)
    return out


def ring_slice_elems(n, count):
    """Elements per owner slice of the bulk kernels' geometry (BulkGeom: ceil(S / n) rounded up to 16 B)."""
    return ((count * 4 + n - 1) // n + 15) // 16 * 4


def ring_order_mismatches(out, n, seq, order="ring"):
    """Elements of a 4-byte-per-element AllReduce output `out` (fp32, ring_tensor inputs of every rank
    for `seq`) that differ bit-wise from the order-stable sum of allreduce_rsag.cu:85-94 / allreduce_rsag_
    zero_copy.cu:88-98: in owner o's slice, x_o + x_{o+1} + ... + x_{o-1}, computed here elementwise by
    torch on out's device in the same order (IEEE fp32 adds, so 0 ulp is the bar).  order="ascending"
    sums x_0 + x_1 + ... instead (tests: a wrong order must be caught)."""
    count = out.numel()
    se = ring_slice_elems(n, count)
    bad = 0
    ov = out.view(torch.int32)
    for o in range(n):
        lo, hi = o * se, min(count, (o + 1) * se)
        for a in range(lo, hi, RING_CHUNK):
            b = min(hi, a + RING_CHUNK)
            ranks = [(o + k) % n for k in range(n)] if order == "ring" else list(range(n))
            acc = ring_tensor(a, b - a, ranks[0], seq, out.device)
            for r in ranks[1:]:
                acc += ring_tensor(a, b - a, r, seq, out.device)
            bad += int((acc.view(torch.int32) != ov[a:b]).sum().item())
    return bad


def ring_oracle_sample(out, n, seq, samples=1 << 16, rng_seed=5):
    """`samples` random elements plus both ends of every owner slice of `out` against the CPU oracle's
    fp32 sum (oracle_reduce_seq, oracle/ll_oracle.c) in ring order from the owner; True if all match."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O

    count = out.numel()
    se = ring_slice_elems(n, count)
    rng = np.random.default_rng(rng_seed)
    idx = np.concatenate([rng.integers(0, count, samples),
                          np.array([v for k in range(n) for v in (k * se, min(count, (k + 1) * se) - 1) if v < count])])
    idx = np.unique(idx).astype(np.int64)
    got = out.view(torch.int32)[torch.from_numpy(idx).to(out.device)].cpu().numpy().view(np.uint32)
    vals = [ring_bits(idx, r, seq).astype(np.int32).view(np.uint32) for r in range(n)]
    owner = idx // se
    for o in range(n):
        sel = owner == o
        if not sel.any():
            continue
        exp = O.reduce_seq(O.F32, O.SUM, [vals[(o + k) % n][sel] for k in range(n)])
        if not np.array_equal(exp, got[sel]):
            return False
    return True


class BitExactChecker:
    """Expected AllReduce results from the CPU oracle (tests/oracle_lib.py -> oracle/liboracle.so) in the sum order
    of the algorithm that produced them; computed lazily, cached per (order, ownership, seq).  Runs outside every
    timed region."""

    def __init__(self, n, S, dt_code):
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib as O

        self.O, self.n, self.S, self.dt = O, n, S, dt_code
        self.inputs = {}
        self.cache = {}

    def _ins(self, seq, nbytes):
        key = (seq, nbytes)
        if key not in self.inputs:
            O = self.O
            self.inputs[key] = [O.lcg(self.dt, nbytes // O.itemsize(self.dt), r, seq) for r in range(self.n)]
        return self.inputs[key]

    def expected(self, algo, nb, nt, seq, nbytes=None, rank=0):
        import mscclpp_amd as m

        O, n = self.O, self.n
        S = nbytes or self.S
        count = S // O.itemsize(self.dt)
        ins = self._ins(seq, S)
        if algo in ("packet", "allpair"):
            # one-hop LL8 (allpair): every rank sums all inputs itself, own first, so the ranks' fp16
            # results differ from each other for n > 2; two-hop LL16 (packet): the owner's sum everywhere
            key = (algo, seq, S, rank)
            if key not in self.cache:
                code = m.ALGO_PACKET if algo == "packet" else m.ALGO_ALLPAIR
                half = m.scratch_required(code, n, S, self.dt) // 2
                fn = O.allreduce_packet if algo == "packet" else O.allreduce_allpairs
                outs, _ = fn(self.dt, O.SUM, ins, count, 1, half)
                self.cache[key] = outs[rank][: (S + 3) // 4].copy()
            return self.cache[key]
        nw = (S + 15) // 16 * 4
        if algo == "rsag_pipeline":
            C = (nb or 32) * (nt or 512) * 4  # units of 16 B per slot and iteration
            chunk, order = 4 * C, 1
        else:
            slice_w = ((S + n - 1) // n + 15) // 16 * 4  # BulkGeom slice (multiple of 16 B)
            chunk, order = slice_w, (0 if algo == "fullmesh" else 1)
        key = (chunk, order, seq, S)
        if key not in self.cache:
            self.cache[key] = O.allreduce_owned(self.dt, O.SUM, ins, nw, n * chunk, chunk, order)[: S // 4]
        return self.cache[key]

    def forget(self):
        """Drop the cached inputs and expectations (host memory: 8 ranks x 256 MiB per size otherwise)."""
        self.inputs.clear()
        self.cache.clear()

    @staticmethod
    def words(t):
        return t.detach().contiguous().view(torch.uint8).cpu().numpy().view(np.uint32)


def bench_multi(args):
    import torch.distributed as dist

    import mscclpp_amd as m

    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    # CPU baselines first, on rank 0 before this process touches a GPU (the other ranks wait in the
    # rendezvous below): the reference's host-proxy path (config 1, its own two processes) and the
    # oracle's n-way sum of the bucket on this box's cores
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        # one proxy rank per GPU; a box with fewer GPUs than ranks (a rehearsal) keeps config 1's two
        # ranks -- eight busy-polling proxy processes spinning kernels on one GPU do not finish
        n_hp = world if torch.cuda.device_count() >= world else 2
        progress(f"CPU baselines: host-proxy loop on {n_hp} ranks")
        hp = host_proxy_baseline(n_hp, timeout=120)
        progress("CPU baselines: oracle n-way sum")
        cpu = {"host_proxy": hp, "sum": cpu_baseline_sum(world, args.bytes, args.cpu_seconds)}
    ndev = torch.cuda.device_count()
    if ndev < world:  # rehearsal on a smaller box: ranks share devices (never the case on the 8-GPU node)
        local = local % ndev
    torch.cuda.set_device(local)
    # a rank that stalls must turn into an error (caught per extras section) well before the driver's
    # limit, so the JSON line is still printed: bounded bootstrap and gloo timeouts
    os.environ.setdefault("MSCCLPP_AMD_BOOTSTRAP_TIMEOUT_S", "180")
    import datetime

    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=600))
    comm = m.Communicator.from_torch_dist()
    n = world
    S = args.bytes
    count = S // 2
    dev = torch.device("cuda", local)
    # two input buffers, LCG seq 0 and 1 (per rank); consecutive steps alternate between them, so a
    # stale output line or a stale scratch line from the previous step never holds the right value
    xs = [lcg_tensor(count, rank, seq, torch.float16, dev) for seq in (0, 1)]
    out = torch.empty_like(xs[0])
    checker = None if args.no_check else BitExactChecker(n, S, m.F16)

    def tmax(v):
        t = torch.tensor([v], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t[0])

    def all_ok(ok):
        t = torch.tensor([1 if ok else 0], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t[0])

    def poison(t):
        t.view(torch.int16).fill_(-1)  # 0xFFFF: an fp16 NaN no correct sum of the LCG inputs produces

    def device_matches(o, exp):
        """The same comparison read by a KERNEL on this rank (through its L2), not by the copy engine:
        peers' remote stores into this rank's output must be what its next kernel reads, with no
        stale L2 line left over from the poison fill."""
        want = torch.from_numpy(exp.view(np.int32).copy()).to(dev)
        flat = o.detach().contiguous().view(torch.uint8)[: want.numel() * 4].view(torch.int32)
        return bool(torch.equal(flat, want))

    def expected_of(algo, nb, nt, nbytes):
        """The oracle's seq-1 result for this rank; algo None = what ncclAllReduce with no algorithm
        runs at this size (the library's selector and its tuned launch shape)."""
        if algo is None:
            algo = SELECT_NAMES[m.lib().mscclppAmdSelectAlgo(n, nbytes or S, 0)]
            nb, nt = _builtin_shape(m, n, nbytes or S)
        return checker.expected(algo, nb, nt, 1, nbytes, rank)

    def verify(o, exp, what):
        """Every word of `o` equals `exp` -- read by the copy engine and by a kernel on this rank --
        and no device error; the verdict of all ranks (MIN), so every rank returns the same."""
        got = BitExactChecker.words(o)
        same = bool(np.array_equal(got, exp)) and device_matches(o, exp)
        if not same:  # say where on stderr (the JSON line carries the verdict per case)
            bad = np.nonzero(got != exp)[0]
            sw = ((got.size * 4 + n - 1) // n + 15) // 16 * 4
            first = int(bad[0]) if bad.size else -1
            print(f"bench: rank {rank} {what}: {bad.size} of {got.size} words differ, first {first} "
                  f"(slice {first // sw}), slices {sorted(set((bad // sw).tolist()))[:8]}, "
                  f"{int((got[bad] == 0xFFFFFFFF).sum())} poisoned", file=sys.stderr)
        return all_ok(same and comm.device_error() == 0)

    def check_run(algo, nb, nt, nbytes=None, bufs=None):
        """Untimed: run once on seq 0, poison the output, run on seq 1, compare every word with the
        oracle.  algo None calls ncclAllReduce with no algorithm (the drop-in caller's path); bufs =
        (seq-0 input, seq-1 input, output) of nbytes when the caller times the same buffers."""
        if bufs is not None:
            a0, a1, o = bufs
        elif nbytes is None:
            a0, a1, o = xs[0], xs[1], out
        else:
            c = nbytes // 2
            a0, a1 = (lcg_tensor(c, rank, sq, torch.float16, dev) for sq in (0, 1))
            o = torch.empty_like(a0)

        def call(a):
            if algo is None:
                comm.all_reduce(a, o)
            else:
                comm.all_reduce(a, o, algo=algo, nblocks=nb, nthreads=nt)

        call(a0)
        poison(o)
        call(a1)
        torch.cuda.synchronize()
        return verify(o, expected_of(algo, nb, nt, nbytes), f"{algo or 'selector'} {nb}x{nt} {nbytes or S} B")

    def check_replay(graph, inp, seq1, o, nbytes):
        """A captured graph reads its input at replay time: load the seq-1 input, poison the output,
        replay once, and compare with the oracle (ncclAllReduce with no algorithm was captured)."""
        inp.copy_(seq1)
        poison(o)
        torch.cuda.synchronize()
        dist.barrier()
        graph.replay()
        torch.cuda.synchronize()
        return verify(o, expected_of(None, 0, 0, nbytes), f"graph replay {nbytes} B")

    vf = None if checker is None else {"check_run": check_run, "check_replay": check_replay, "poison": poison,
                                       "all_ok": all_ok, "forget": checker.forget}

    # ---- the built-in selector's choice, as a drop-in caller of ncclAllReduce gets it before any
    # tuning (algo None -> ncclAllReduce -> mscclppAmdSelectAlgo + its launch shape), timed like the
    # headline: the `default_selector` figure beside it
    progress("default selector")
    default_sel = {"algo": SELECT_NAMES[m.lib().mscclppAmdSelectAlgo(n, S, 0)],
                   "source": m.tuned_config_source("allreduce", n, S)}
    try:
        for j in range(3):
            comm.all_reduce(xs[j % 2], out)
        torch.cuda.synchronize()
        dist.barrier()
        td = tmax(_time_calls(lambda: comm.all_reduce(xs[0], out), max(5, min(args.steps, 20))))
        default_sel.update({"ms_per_step": round(td * 1e3, 4), "algbw_GBs": round(S / td / 1e9, 2),
                            "frac_of_assumed_ceiling": round(S / td / 1e9 / (n * XGMI_LINK_GBS / 2), 4),
                            "correct_bitexact": check_run(default_sel["algo"], *_builtin_shape(m, n, S))
                            if checker is not None else None})
    except Exception as e:  # recorded, never fatal for the headline line
        default_sel["error"] = str(e)[-300:]
    # ---- pick the algorithm and launch shape (untimed; every rank tries the same candidates in the
    # same order).  Large buckets: the scratch-based all-pairs RS+AG (fullmesh, puts), the zero-copy
    # RS+AG (reads peers' inputs, writes peers' outputs) and the pipelined RS+AG -- which one drives
    # xGMI best is measured here, on the node, not assumed.
    sel = SELECT_NAMES[m.lib().mscclppAmdSelectAlgo(n, S, 0)]
    algos = [args.algo] if args.algo else ([sel] + [a for a in ("fullmesh", "rsag_zc", "rsag_pipeline") if a != sel]
                                           if sel in ("fullmesh", "rsag_zc", "rsag_pipeline") else [sel])
    cands = []
    shared = ndev_shared(world)  # rehearsal: ranks share a device, so every rank's grid must fit on it at once
    # rehearsal shapes: small enough that every rank's grid is resident on the one shared device
    bulk_shapes = ((32, 512), (64, 512), (128, 512), (256, 512), (128, 256), (256, 256)) if not shared else \
        tuple((nb_, 512) for nb_ in (16, 32, 64, 128) if nb_ * world <= 256)
    pipe_shapes = ((32, 512), (64, 512), (128, 512), (64, 256)) if not shared else \
        tuple((nb_, 512) for nb_ in (8, 16, 32, 64) if 2 * nb_ * world <= 256)
    for a in algos:
        if a in ("fullmesh", "rsag", "rsag_zc"):
            cands += [(a, nb_, nt_) for nb_, nt_ in bulk_shapes]
        elif a == "rsag_pipeline":  # nblocks = reduce workgroups; the launch is 2x that
            cands += [(a, nb_, nt_) for nb_, nt_ in pipe_shapes]
        else:
            cands.append((a, 0, 0))
    if not cands:
        raise SystemExit(f"bench: no launch shape fits {world} ranks on {ndev} device(s)")
    tune = {}
    progress(f"tuning {len(cands)} candidates")
    for a, nb, nt in cands:
        try:
            for j in range(2):
                comm.all_reduce(xs[j], out, algo=a, nblocks=nb, nthreads=nt)
            torch.cuda.synchronize()
            dist.barrier()  # the ranks start each candidate's timed calls together
            tune[(a, nb, nt)] = tmax(_time_calls(lambda: comm.all_reduce(xs[0], out, algo=a, nblocks=nb, nthreads=nt), 5))
        except Exception as e:  # a rejected shape is simply skipped
            tune[(a, nb, nt)] = float("inf")
            if rank == 0:
                print(f"tune {a} {nb}x{nt}: {e}", file=sys.stderr)
    if tmax(float(comm.device_error())) != 0:  # a spin timed out somewhere: say so instead of hanging on
        print("bench: device error after tuning; results below are suspect", file=sys.stderr)
    algo, nb, nt = min(tune, key=tune.get)
    # ---- the winner goes into the library's own selector (mscclppAmdTunedConfigLoad, the tuned-config
    # store of host/tuning.cpp), and the timed region calls ncclAllReduce with no algorithm and no
    # launch shape, exactly as a drop-in caller does (nccl.cc:607-660 -> algorithm_selector.cc:91-139)
    loaded = load_winner(m, n, S, torch.cuda.get_device_name(dev), algo, nb, nt)
    sel_algo = SELECT_NAMES[m.lib().mscclppAmdSelectAlgo(n, S, 0)]
    sel_shape = m.tuned_config("allreduce", n, S)
    if sel_algo != algo or sel_shape is None or tuple(sel_shape[1:]) != (nb, nt):
        raise SystemExit(f"bench: the loaded tuned config selects {sel_algo} {sel_shape}, not {algo} {nb}x{nt}")

    total = args.warmup + args.steps

    def step(j):  # step j of warmup + timed; the last timed step runs on seq 1 -- ncclAllReduce
        comm.all_reduce(xs[1 if args.same_input else 1 - (total - 1 - j) % 2], out)

    progress(f"selected {algo} {nb}x{nt}; warmup + timed region")
    poison(out)  # the fill kernel's first launch loads its code object (~4 ms): never inside the timed region
    for j in range(args.warmup):
        step(j)
    torch.cuda.synchronize()
    # ---- timed region: exactly K steps, barrier + synchronize on both sides, max over ranks; the
    # kernel duration from an event pair on the launch stream around the same K launches.  The output
    # is poisoned (one fill) before the last step, whose result is then checked bit-exactly.
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record()
    for j in range(args.warmup, total):
        if j == total - 1:
            poison(out)
        step(j)
    ev1.record()
    torch.cuda.synchronize()
    t_local = (time.perf_counter() - t0) / args.steps
    dist.barrier()
    t = tmax(t_local)
    kern_ms = tmax(ev0.elapsed_time(ev1) / args.steps)
    errc = comm.device_error()
    bitexact = {}
    if checker is not None:
        progress("bit-exact check of the timed step and of every tuned candidate")
        exp = checker.expected(algo, nb, nt, 1, None, rank)
        bitexact["timed_last_step"] = all_ok(bool(np.array_equal(BitExactChecker.words(out), exp))
                                             and device_matches(out, exp) and errc == 0)
        for a, cnb, cnt in cands:
            if tune[(a, cnb, cnt)] == float("inf"):
                continue
            bitexact[f"{a}:{cnb}x{cnt}"] = check_run(a, cnb, cnt)
        # in place (send == recv, BASELINE configs[2] names both): the winner once more
        a1 = xs[1].clone()
        comm.all_reduce(a1, a1, algo=algo, nblocks=nb, nthreads=nt)
        torch.cuda.synchronize()
        exp1 = checker.expected(algo, nb, nt, 1, None, rank)
        bitexact[f"{algo}:{nb}x{nt}:in_place"] = all_ok(bool(np.array_equal(BitExactChecker.words(a1), exp1))
                                                        and device_matches(a1, exp1) and comm.device_error() == 0)
        del a1
        for a, nbytes in (("packet", 1 << 20), ("allpair", 16 << 10)):  # the LL paths (configs[3])
            try:
                bitexact[f"{a}:{nbytes >> 10}KiB"] = check_run(a, 0, 0, nbytes)
            except Exception as e:  # recorded, never fatal for the headline line
                bitexact[f"{a}:{nbytes >> 10}KiB"] = f"error: {e}"[:200]
    phases = phase_breakdown(m, comm, n, dev, tmax, algo, nb, nt, xs[0], out)
    ok = errc == 0 and all(v is True for v in bitexact.values()) if bitexact else errc == 0
    if not bitexact:  # --no-check: fp32 gloo reference with the tolerance of correctness.py:257-258
        ref = xs[1].float().cpu()
        dist.all_reduce(ref)
        ok = bool(torch.allclose(out.float().cpu(), ref, rtol=1e-2, atol=5e-4 * n)) and errc == 0
    algbw = S / t / 1e9
    progress("xGMI probe")
    try:
        probe = xgmi_probe(comm, n, dev, tmax, dist.barrier)
    except Exception as e:  # recorded, never fatal for the headline line
        probe = {"error": str(e)[-300:]}
    roofline, xgmi = multi_roofline(n, S, algo, t, kern_ms, probe, ndev < world)
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
        "data": "synthetic (LCG of test/torch/correctness_test.py, seq alternating per step)",
        "config": {"workload": f"allreduce_fp16_{S >> 20}MiB (BASELINE configs[2]: 2048x12288 fp16 bucket per rank)",
                   "bytes": S, "parallelism": f"allreduce{world}", "call": "ncclAllReduce (algorithm and shape "
                   "from the library's selector after mscclppAmdTunedConfigLoad of this node's winner)",
                   "algo": sel_algo, "nblocks": nb, "nthreads": nt, "tuned_config_loaded": loaded,
                   "selector_source": m.tuned_config_source("allreduce", n, S)},
        "default_selector": default_sel,
        # ranks sharing fewer GPUs than ranks (a 1-GPU box): every number below is HBM, not xGMI
        "rehearsal": ndev < world,
        "scaling_note": SCALING_NOTE,
        "busbw": round(algbw * 2 * (n - 1) / n, 2),
        # the bytes all ranks contributed per AllReduce (n buckets of S) over the step time, beside
        # the metric's algbw (S / t, one bucket per collective, nccl-tests' convention)
        "aggregate_input_GBs": round(n * S / t / 1e9, 2),
        "roofline": roofline,
        "xgmi": xgmi,
        "tune_ms": {f"{k[0]}:{k[1]}x{k[2]}": round(v * 1e3, 4) for k, v in tune.items()},
        "correct": ok,
        "correct_bitexact": bitexact,
        "phases_us": phases,
    }
    # the winner in the tuned-config format of python/mscclpp_benchmark/tuning_config.py, to be loaded
    # with MSCCLPP_AMD_TUNED_CONFIG (or merged into the built-in table, host/tuning.cpp)
    res["tuned_config"] = {"version": 1, "profiles": [{"sku": torch.cuda.get_device_name(dev), "scale": n,
                                                       "collectives": {"allreduce": [
                                                           {"message_size": S, "algorithm": FULL_NAMES[algo],
                                                            "nblocks": nb, "nthreads": nt,
                                                            "time_us": round(t * 1e6, 2)}]}}]}
    if cpu is not None:
        hp = cpu["host_proxy"]
        res["cpu_baseline"] = dict(cpu["sum"])
        res["host_proxy_baseline"] = hp
    if not args.no_extras:
        res["extras"] = bench_extras(args, comm, n, dev, tmax, dist.barrier, vf)
        # every size and kernel the extras time is checked first (mscclpp-test common.cc:346-360
        # checks each size it times): all of those verdicts, and any section that failed, are part
        # of `correct`
        res["correct"] = bool(res["correct"] and extras_correct(res["extras"], vf is not None))
        # every measured winner as a ready-to-commit tuned-config profile for this node and scale --
        # only from a node where every rank has its own GPU; a rehearsal's table is tagged as such
        table = node_tuned_table(n, torch.cuda.get_device_name(dev), res["extras"], (S, algo, nb, nt))
        if ndev < world:
            res["tuned_config_table_rehearsal"] = dict(table, rehearsal=True)
        else:
            res["tuned_config_table"] = table
    # last: on a rehearsal box (ranks sharing one device) the extra stream queues of a graph capture
    # slow every later launch of those ranks, so nothing is measured after it
    progress("graph-captured headline")
    try:
        # common.cc:202-227: 20 calls captured in one graph, 15 graph launches, per-call time
        g_s, graph = graph_time_per_call(lambda: comm.all_reduce(xs[0], out),
                                         calls=20, replays=15, sync=dist.barrier, keep=True)
        g_s = tmax(g_s)
        res["graph"] = {"us_per_call": round(g_s * 1e6, 2), "algbw_GBs": round(S / g_s / 1e9, 2),
                        "note": "20 calls per HIP graph, 15 launches (mscclpp-test common.cc:202-227); value stays the eager loop"}
        if checker is not None:  # a replay reads the input as it is at replay time: new data, poisoned output
            xs[0].copy_(xs[1])
            poison(out)
            torch.cuda.synchronize()
            dist.barrier()
            graph.replay()
            torch.cuda.synchronize()
            exp = checker.expected(algo, nb, nt, 1, None, rank)
            res["graph"]["replay_bitexact"] = all_ok(bool(np.array_equal(BitExactChecker.words(out), exp))
                                                     and device_matches(out, exp) and comm.device_error() == 0)
            res["correct"] = bool(res["correct"] and res["graph"]["replay_bitexact"])
        del graph
    except Exception as e:  # recorded, never fatal for the headline line
        res["graph"] = {"error": str(e)[-300:]}
    comm.destroy()
    dist.barrier()
    dist.destroy_process_group()
    return res if rank == 0 else None


def _builtin_shape(m, n, S):
    """(nblocks, nthreads) the library's selector gives an AllReduce of S bytes (0 = kernel default)."""
    t = m.tuned_config("allreduce", n, S)
    return (t[1], t[2]) if t else (0, 0)


def winner_profile(m, n, S, sku, algo, nb, nt):
    """A tuned-config store (python/mscclpp_benchmark/tuning_config.py format) for this SKU and rank
    count that keeps the selector's current choices below the bucket -- the LL thresholds at 1 B,
    16 KiB + 1 and 1 MiB + 1 -- and names the tuned winner from S up.  Computed before it is loaded."""
    entries = []
    for size in (1, (16 << 10) + 1, (1 << 20) + 1):
        if size >= S:
            break
        a = SELECT_NAMES[m.lib().mscclppAmdSelectAlgo(n, size, 0)]
        nb_, nt_ = _builtin_shape(m, n, size)
        e = {"message_size": size, "algorithm": FULL_NAMES[a], "nblocks": nb_, "nthreads": nt_,
             "source": m.tuned_config_source("allreduce", n, size)}
        if not entries or {k: v for k, v in entries[-1].items() if k != "message_size"} != \
                {k: v for k, v in e.items() if k != "message_size"}:
            entries.append(e)
    entries.append({"message_size": S, "algorithm": FULL_NAMES[algo], "nblocks": nb, "nthreads": nt,
                    "source": "tuned (bench.py, this run)"})
    prof = {"scale": n, "collectives": {"allreduce": entries}}
    if sku:
        prof = {"sku": sku, **prof}
    return {"version": 1, "profiles": [prof]}


def load_winner(m, n, S, sku, algo, nb, nt):
    """Write winner_profile to a file and load it into the library (mscclppAmdTunedConfigLoad)."""
    import tempfile

    prof = winner_profile(m, n, S, sku, algo, nb, nt)
    with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as f:
        json.dump(prof, f)
        path = f.name
    try:
        m.load_tuned_config(path)
    finally:
        os.unlink(path)
    return prof["profiles"][0]["collectives"]["allreduce"]


def multi_roofline(n, S, algo, t, kern_ms, probe, rehearsal):
    """The N>1 line's `roofline` and `xgmi` objects, graded against north_star's target (>= 80 % of
    aggregate xGMI algorithm bandwidth).  peak = the all-pairs AllReduce algbw ceiling of BASELINE.md
    §2 / SURVEY §8(d) config 3 at the task-stated link rate, n * 153.6 / 2 GB/s (614.4 at n = 8):
    every rank moves 2(n-1)/n * S over its n-1 links of 153.6 GB/s.  achieved = S / the dominant
    kernel's average launch time, so frac = achieved / peak, equivalently its wire bytes per rank
    over (n-1) * 153.6 GB/s.  The same run's raw-access probe of the kernel's own pattern (zero-copy:
    all-pairs gets + puts in one launch, allreduce_rsag_zero_copy.cu:88-92; the scratch kernels:
    all-pairs puts) is reported beside it as measured_ceiling / frac_of_measured -- never the peak,
    which would grade the kernel against itself.  An AllReduce cannot move its bytes faster than the
    raw accesses it is made of, so a frac_of_measured above 1 sets probe_consistent false."""
    algbw = S / t / 1e9
    peak = n * XGMI_LINK_GBS / 2  # all-pairs algbw ceiling at the assumed link rate
    kern_algbw = S / (kern_ms * 1e-3) / 1e9
    wire = 2 * (n - 1) * S / n
    wire_ach = wire / (kern_ms * 1e-3) / 1e9
    # HBM bytes one rank's AllReduce moves.  fullmesh/rsag: reads S input + (n-1)/n S scratch;
    # writes S/n own output + (n-1)/n S incoming scratch + (n-1)/n S incoming output.  rsag_zc: reads
    # S of input (own slice locally, the rest by the peers), writes S of output (own slice locally,
    # the rest by the peers).  rsag_pipeline: reads S input + 2(n-1)/n S scratch (RS and AG regions),
    # writes S output + 2(n-1)/n S incoming scratch
    hbm = (2 * S if algo == "rsag_zc" else 2 * S * (1 + 2 * (n - 1) / n) if algo == "rsag_pipeline"
           else S * (1 + 3 * (n - 1) / n + 1 / n))
    pattern = "allpairs_getput_GBs" if algo == "rsag_zc" else "allpairs_put_out_GBs"
    raw = probe.get(pattern)  # wire GB/s per rank of the kernel's access pattern, this run
    kernel = {"rsag_zc": "allreduceZeroCopyKernel", "rsag_pipeline": "allreduceRsAgPipelineKernel",
              "packet": "allreduceLL16Kernel", "allpair": "allreduceLL8Kernel"}.get(algo, f"allreduceBulkKernel ({algo})")
    roofline = {"bound": "xgmi", "achieved": round(kern_algbw, 1), "peak": round(peak, 1), "unit": "GB/s",
                "frac": round(kern_algbw / peak, 4), "traffic": None,
                "peak_source": "BASELINE.md §2 all-pairs AllReduce algbw ceiling n * 153.6 / 2 GB/s (n - 1 xGMI "
                               "links of 153.6 GB/s per GPU, 2(n-1)/n * S wire bytes per rank)",
                "achieved_note": "S / average launch time of the dominant kernel (HIP events on its stream); "
                                 "frac = wire bytes per rank / ((n-1) * 153.6 GB/s), the same number",
                "rehearsal": bool(rehearsal),
                "wire_GBs_per_rank": round(wire_ach, 1), "wire_peak_GBs_per_rank": round((n - 1) * XGMI_LINK_GBS, 1),
                "kernel": kernel, "kernel_us": round(kern_ms * 1e3, 2),
                "algorithmic_bytes_per_launch": int(S), "wire_bytes_per_rank_per_launch": int(wire),
                "hbm": {"achieved": round(hbm / (kern_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                        "frac": round(hbm / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                        "bytes_per_launch": int(hbm)},
                # traffic stays null: no counters run on the node.  The committed fabric-free PMC
                # run of the same kernel (8 in-process ranks) gives its bytes over its algorithmic ones
                "pmc_fabric_free": committed_multirank_pmc(kernel)}
    xgmi = {"allpairs_algbw_ceiling_assumed": round(peak, 1), "frac_of_assumed_ceiling": round(algbw / peak, 4),
            "link_GBs_assumed": XGMI_LINK_GBS, "wire_bytes_per_rank": int(wire), "measured": probe}
    if raw:
        mc = raw * n / (2 * (n - 1))  # algbw ceiling: 2(n-1)/n * S wire bytes per AllReduce at that rate
        roofline["measured_ceiling"] = round(mc, 1)
        roofline["frac_of_measured"] = round(kern_algbw / mc, 4)
        roofline["measured_ceiling_source"] = (f"xgmi_probe.{pattern} = {raw} GB/s per rank: raw accesses of the "
                                               "kernel's own remote pattern, one launch in this run, as algbw")
        xgmi["allpairs_algbw_ceiling_measured"] = round(mc, 1)
        xgmi["frac_of_measured_ceiling"] = round(algbw / mc, 4)
        xgmi["probe_consistent"] = bool(wire_ach <= raw and algbw <= mc)
    else:
        xgmi["probe_consistent"] = False
    return roofline, xgmi


def phase_breakdown(m, comm, n, dev, tmax, algo, nb, nt, x, out):
    """Where the time of one call goes, per kernel phase (the NPKit role; m.PhaseTrace): the
    headline winner at its shape and the two LL paths of configs[3] (1 MiB LL16, 16 KiB LL8).  Four
    calls run back to back with the trace on, so the stamped (last) call starts when its
    predecessor's handshakes released every rank; each phase's mean and max over workgroups, then
    the max over ranks.  Untimed, after the headline; failures are recorded, not raised."""
    res = {}
    for a, nb_, nt_, nbytes in ((algo, nb, nt, None), ("packet", 0, 0, 1 << 20), ("allpair", 0, 0, 16 << 10)):
        if a not in m.TRACE_PHASES:
            continue
        key = f"{a}:{nb_}x{nt_}" if nbytes is None else f"{a}:{nbytes >> 10}KiB"
        try:
            xi, oi = (x, out) if nbytes is None else (x[: nbytes // 2], out[: nbytes // 2])
            comm.all_reduce(xi, oi, algo=a, nblocks=nb_, nthreads=nt_)
            torch.cuda.synchronize()
            with m.PhaseTrace(dev) as tr:
                for _ in range(4):
                    comm.all_reduce(xi, oi, algo=a, nblocks=nb_, nthreads=nt_)
            ph = tr.phases(a)
            row = {}
            for name in m.TRACE_PHASES[a]:
                v = ph.get(name, {"mean_us": 0.0, "max_us": 0.0})
                row[name] = {"mean_us": round(tmax(v["mean_us"]), 2), "max_us": round(tmax(v["max_us"]), 2)}
            row["kernel_span_us"] = round(tmax(ph.get("kernel_span_us", 0.0)), 2)
            row["workgroups"] = ph.get("workgroups", 0)
            res[key] = row
        except Exception as e:  # noqa: BLE001
            res[key] = {"error": str(e)[-200:]}
    return res


def xgmi_probe(comm, n, dev, tmax, barrier, S=64 << 20):
    """Raw xGMI ceilings measured on the node (calibrate B_link with a raw put
    microbenchmark), each as ONE launch of mscclppAmdCopyJobs on one stream (workgroups partitioned by
    peer, 16-byte system-scope loads/stores; GPU_MAX_HW_QUEUES does not limit it):
      ring_put       every rank writes S into the next rank (each link carries one direction)
      ring_get       every rank reads S from the previous rank
      allpairs_put   every rank writes S/(n-1) into each peer at once (all 7 links out, the AllReduce's
                     RS / AG pattern); GB/s = bytes out per rank / time
      allpairs_get   every rank reads S/(n-1) from each peer at once
    Max time over ranks, 5 launches each after a warm-up."""
    import mscclpp_amd as m

    L = m.lib()
    rank = comm.rank
    src = torch.full((S,), rank & 0xFF, dtype=torch.uint8, device=dev)
    dst = torch.empty(S, dtype=torch.uint8, device=dev)
    pdst = comm.register_buffer(dst)
    psrc = comm.register_buffer(src)
    nxt, prv = (rank + 1) % n, (rank - 1) % n
    vp, sz = ctypes.c_void_p, ctypes.c_size_t

    def jobs(pairs, bpj, lp=0, sp=0):
        k = len(pairs)
        srcs = (vp * k)(*[p[0] for p in pairs])
        dsts = (vp * k)(*[p[1] for p in pairs])
        lens = (sz * k)(*[p[2] for p in pairs])
        return lambda: m.check(L.mscclppAmdCopyJobsPolicy(srcs, dsts, lens, k, bpj, lp, sp, m.stream_ptr()),
                               "copy jobs")

    def timed(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return tmax((time.perf_counter() - t0) / reps)

    base_s, base_d = src.data_ptr(), dst.data_ptr()
    # one link at a time: every rank puts S/4 into the peer at distance d (d = 1 .. n-1) in the same
    # launch, so each rank drives exactly one outgoing link and receives on one; a node whose links
    # differ (topology, a degraded link) shows it here
    per_peer = {}
    for d in range(1, n):
        q = (rank + d) % n
        per_peer[f"+{d}"] = round((S // 4) / timed(jobs([(base_s, pdst[q], S // 4)], 512)) / 1e9, 1)
    t_put = timed(jobs([(base_s, pdst[nxt], S)], 512))
    t_get = timed(jobs([(psrc[prv], base_d, S)], 512))
    chunk = (S // (n - 1)) // 16 * 16
    peers = [q for q in range(n) if q != rank]
    bpj = max(32, 1024 // (n - 1))
    # distinct destination region per (source, destination): slot = position of the source among the
    # destination's peers, so no two writers share a region
    put = [(base_s + i * chunk, pdst[q] + ((rank - q - 1) % n) * chunk, chunk) for i, q in enumerate(peers)]
    get = [(psrc[q] + ((q - rank - 1) % n) * chunk, base_d + i * chunk, chunk) for i, q in enumerate(peers)]
    t_ap = timed(jobs(put, bpj))
    t_ag = timed(jobs(get, bpj))
    # the zero-copy pattern: gets from every peer and puts into every peer in ONE launch, the gets
    # landing in a buffer of their own (bytes in + bytes out per rank over the time)
    gdst = torch.empty(S, dtype=torch.uint8, device=dev)
    getput = [(psrc[q] + ((q - rank - 1) % n) * chunk, gdst.data_ptr() + i * chunk, chunk) for i, q in enumerate(peers)]
    t_gp = timed(jobs(put + getput, max(16, bpj // 2)))
    del gdst
    # what the cache policy of the remote accesses costs over the links (the collectives use sc0 sc1
    # everywhere): all-pairs puts by store policy, all-pairs gets by load policy
    pol = {"sys": 0, "plain": 1, "nt": 2, "agent": 3}
    by_store = {k: round((n - 1) * chunk / timed(jobs(put, bpj, 0, v)) / 1e9, 1) for k, v in pol.items()}
    by_load = {k: round((n - 1) * chunk / timed(jobs(get, bpj, v, 0)) / 1e9, 1) for k, v in pol.items()}
    barrier()
    out = {"bytes": S, "launch": "mscclppAmdCopyJobs, one stream", "ring_put_GBs": round(S / t_put / 1e9, 1),
           "ring_get_GBs": round(S / t_get / 1e9, 1),
           "allpairs_put_out_GBs": round((n - 1) * chunk / t_ap / 1e9, 1),
           "allpairs_get_in_GBs": round((n - 1) * chunk / t_ag / 1e9, 1),
           "allpairs_getput_GBs": round(2 * (n - 1) * chunk / t_gp / 1e9, 1),
           "allpairs_put_out_GBs_by_store_policy": by_store, "allpairs_get_in_GBs_by_load_policy": by_load,
           "single_link_put_GBs_by_distance": per_peer}
    # all-pairs AllReduce moves 2(n-1)/n * S per rank: its algbw ceilings at the measured rates
    out["allpairs_algbw_ceiling_put"] = round(out["allpairs_put_out_GBs"] * n / (2 * (n - 1)), 1)
    out["allpairs_algbw_ceiling_getput"] = round(out["allpairs_getput_GBs"] * n / (2 * (n - 1)), 1)
    del pdst, psrc
    return out


def graph_time_per_call(fn, calls=20, replays=10, sync=None, keep=False):
    """Per-call time with `calls` calls captured in one HIP graph (mscclpp-test common.cc:202-227).
    `sync` (a host barrier across ranks) lines the ranks up before the timed replays, so the first
    replay does not absorb another rank's late start.  keep=True: (time, graph)."""
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
    t = _time_calls(g.replay, replays) / calls
    return (t, g) if keep else t


def ndev_shared(n):
    """True in a rehearsal where n ranks share fewer devices, so every rank's grid must fit on the
    device at once and the launch shapes are cut down.  BENCH_NODE_SHAPES=1 (diagnosis) keeps the
    node's shapes anyway: a 2-rank run on one GPU then walks the node-only branches of this file."""
    return torch.cuda.device_count() < n and os.environ.get("BENCH_NODE_SHAPES") != "1"


LL_SWEEP_KIB = tuple(1 << k for k in range(11))  # BASELINE configs[3]: 1 KiB .. 1 MiB, x2 steps
CROSSOVER_KIB = (4, 8, 16, 32, 64, 256, 512, 1024, 2048, 4096)  # both sides of the 16 KiB and 1 MiB thresholds


def node_tuned_table(n, sku, extras, headline):
    """The node's measured winners as one tuned-config profile (python/mscclpp_benchmark/
    tuning_config.py format, loaded by MSCCLPP_AMD_TUNED_CONFIG): per measured message size the
    fastest candidate of the selector-crossover and bulk-size sweeps and the headline's tuning;
    an entry applies from its message_size up to the next one, so runs of one winner collapse."""
    pts = []
    for kb, row in (extras.get("selector_crossover") or {}).items():
        pts.append((int(kb[:-3]) << 10, row["best"]))
    for mb, row in (extras.get("bulk_size_sweep") or {}).items():
        pts.append((int(mb[:-3]) << 20, row["best"]))
    if headline:
        pts.append((headline[0], f"{headline[1]}:{headline[2]}x{headline[3]}"))
    pts.sort(key=lambda p: p[0])  # stable: at a size both sweeps measured, the bulk sweep's row comes last and wins
    if pts:
        pts.insert(0, (1, pts[0][1]))
    entries = []
    for size, key in pts:
        algo, shape = key.split(":")
        nb, nt = (int(v) for v in shape.split("x"))
        e = {"message_size": size, "algorithm": FULL_NAMES[algo], "nblocks": nb, "nthreads": nt,
             "source": f"node ({sku}, {n} ranks, bench.py)"}
        if entries and {k: v for k, v in entries[-1].items() if k != "message_size"} == \
                {k: v for k, v in e.items() if k != "message_size"}:
            continue
        if entries and entries[-1]["message_size"] == size:
            entries[-1] = e
            continue
        entries.append(e)
    return {"version": 1, "profiles": [{"sku": sku, "scale": n, "collectives": {"allreduce": entries}}]}


EXTRAS_CHECK_KEYS = (["ll_sweep:%dKiB" % kb for kb in LL_SWEEP_KIB] + ["ll_graph:%dKiB" % kb for kb in LL_SWEEP_KIB]
                     + ["ll16_48MiB", "fp32_1GiB_rsag", "fp32_1GiB_rsag_zc"])


def extras_correct(extras, checked):
    """True when no extras section failed and (checked) every case of EXTRAS_CHECK_KEYS is present
    in extras["correct_bitexact"] and True; a section's error, or a missing case, is False."""
    if any(k.endswith("_error") and k != "device_error" for k in extras) or extras.get("device_error", 0):
        return False
    if not checked:
        return True
    cb = extras.get("correct_bitexact", {})
    return all(cb.get(k) is True for k in EXTRAS_CHECK_KEYS) and all(v is True for v in cb.values())


def ll16_ceiling(n):
    """The LL16 AllReduce's algbw ceiling over xGMI: the all-pairs ceiling n * 153.6 / 2 GB/s halved,
    since every 16-byte LL16 packet carries 8 bytes of data and two 4-byte flags (SURVEY §7 "LL
    framing"; docs/tutorials/03-memory-channel.md:26-34)."""
    return n * XGMI_LINK_GBS / 4


def bench_extras(args, comm, n, dev, tmax, barrier, vf=None):
    """BASELINE configs[3] (LL latency sweep, fp16 1 KiB..1 MiB, eager and graph-captured), LL16 at
    the headline bucket, and configs[4] (fp32 1 GiB RS+AG in ring order), each size checked
    bit-exactly before it is timed (vf: bench_multi's checkers; None under --no-check); failures are
    recorded, not raised.  Verdicts go to extras["correct_bitexact"]."""
    import mscclpp_amd as m

    extras = {}
    checks = extras["correct_bitexact"] = {}
    rank = comm.rank

    def lcg_pair(cnt):
        return [lcg_tensor(cnt, rank, sq, torch.float16, dev) for sq in (0, 1)]

    progress("extras: LL latency sweep")
    try:
        lat = {}
        for kb in LL_SWEEP_KIB:
            a0, a1 = lcg_pair(kb * 512)
            os_ = torch.empty_like(a0)
            if vf:  # ncclAllReduce with no algorithm, exactly as timed below
                checks[f"ll_sweep:{kb}KiB"] = vf["check_run"](None, 0, 0, kb << 10, bufs=(a0, a1, os_))
            for _ in range(5):
                comm.all_reduce(a1, os_)
            torch.cuda.synchronize()
            barrier()
            lat[f"{kb}KiB"] = round(tmax(_time_calls(lambda: comm.all_reduce(a1, os_), 50)) * 1e6, 2)
        extras["ll_latency_us"] = lat
        extras["ll_latency_algo"] = {f"{kb}KiB": SELECT_NAMES[m.lib().mscclppAmdSelectAlgo(n, kb << 10, 0)]
                                     for kb in LL_SWEEP_KIB}
    except Exception as e:
        extras["ll_latency_error"] = str(e)
    progress("extras: LL16 at the headline bucket")
    try:
        # LL16 two-hop at the 48 MiB bucket, graded against its own halved ceiling;
        # default shape and two wider grids, each checked bit-exactly (owner's sum of
        # allreduce_packet.cu:93-106) before it is timed
        nbytes = args.bytes
        a0, a1 = lcg_pair(nbytes // 2)
        o = torch.empty_like(a0)
        peers = n - 1
        # rehearsals at 2-4 ranks: wider grids win at this size (4 ranks: 48 workgroups 605 us,
        # 96 workgroups 352 us; profiles/r5_bench_n4_rehearsal_line.json), so the node tries up to 64
        # per peer (448 at 8 ranks, all resident on one GPU)
        shapes = [(0, 0), (peers * 16, 512), (peers * 32, 512), (peers * 64, 512)]
        if ndev_shared(n):  # rehearsal: every rank's grid resident on the shared device
            shapes = [s for s in shapes if s[0] * n <= 512]
        row, ok = {}, True
        for nb_, nt_ in shapes:
            key = f"packet:{nb_}x{nt_}"
            try:
                if vf:
                    good = vf["check_run"]("packet", nb_, nt_, nbytes, bufs=(a0, a1, o))
                    ok = ok and good
                    row[key + ":bitexact"] = good
                for _ in range(2):
                    comm.all_reduce(a1, o, algo="packet", nblocks=nb_, nthreads=nt_)
                torch.cuda.synchronize()
                barrier()
                row[key] = round(tmax(_time_calls(
                    lambda: comm.all_reduce(a1, o, algo="packet", nblocks=nb_, nthreads=nt_), 5)) * 1e6, 1)
            except Exception as e:  # noqa: BLE001 -- a shape the library refuses is recorded
                row[key] = str(e)[:80]
                ok = False
        times = [(v, k) for k, v in row.items() if isinstance(v, float)]
        if times:
            best_us, best = min(times)
            ach = nbytes / (best_us * 1e-6) / 1e9
            extras["ll16_48MiB"] = {"bytes": nbytes, "us": row, "best": best, "algbw_GBs": round(ach, 2),
                                    "peak": round(ll16_ceiling(n), 1), "frac": round(ach / ll16_ceiling(n), 4),
                                    "peak_source": "n * 153.6 / 4 GB/s: the all-pairs ceiling halved by LL16 framing "
                                                   "(8 data bytes per 16-byte packet)"}
        if vf:
            checks["ll16_48MiB"] = bool(ok and times)
            vf["forget"]()
        del a0, a1, o
    except Exception as e:
        extras["ll16_48MiB_error"] = str(e)[-300:]
    progress("extras: bulk size sweep")
    try:
        # per message size, the best of the bulk algorithms at two shapes each (fp16): the data for
        # the tuned-config table (host/tuning.cpp) above the LL range
        sweep = {}
        big0, big = lcg_pair((256 << 20) // 2)
        bout = torch.empty_like(big)
        for mb in (2, 4, 8, 16, 32, 64, 128, 256):
            xs, os_ = big[: (mb << 20) // 2], bout[: (mb << 20) // 2]
            row = {}
            shapes = (("fullmesh", 64, 512), ("fullmesh", 128, 512), ("rsag_zc", 64, 512),
                      ("rsag_zc", 128, 512), ("rsag_pipeline", 32, 512), ("rsag_pipeline", 64, 512))
            if ndev_shared(n):  # rehearsal: every rank's grid resident on the shared device
                shapes = tuple((a, max(8, 256 // ((2 if a == "rsag_pipeline" else 1) * n) // k), 512)
                               for a, k in (("fullmesh", 1), ("rsag_zc", 1), ("rsag_pipeline", 1)))
            for a, nb_, nt_ in shapes:
                try:
                    for _ in range(2):
                        comm.all_reduce(xs, os_, algo=a, nblocks=nb_, nthreads=nt_)
                    torch.cuda.synchronize()
                    barrier()
                    row[f"{a}:{nb_}x{nt_}"] = round(tmax(_time_calls(
                        lambda: comm.all_reduce(xs, os_, algo=a, nblocks=nb_, nthreads=nt_), 5)) * 1e6, 1)
                except Exception as e:  # noqa: BLE001
                    row[f"{a}:{nb_}x{nt_}"] = str(e)[:80]
            best = min((v, k) for k, v in row.items() if isinstance(v, float))
            sweep[f"{mb}MiB"] = {"us": row, "best": best[1], "algbw_GBs": round((mb << 20) / best[0] / 1e3, 1)}
            if vf:  # the winner (it goes into the node's tuned table) checked bit-exactly at this size
                a, shp = best[1].split(":")
                nb_, nt_ = (int(v) for v in shp.split("x"))
                checks[f"bulk_sweep:{mb}MiB:{best[1]}"] = vf["check_run"](
                    a, nb_, nt_, mb << 20, bufs=(big0[: (mb << 20) // 2], xs, os_))
                vf["forget"]()
        extras["bulk_size_sweep"] = sweep
        del big0, big, bout
    except Exception as e:
        extras["bulk_size_sweep_error"] = str(e)[-300:]
    progress("extras: selector crossover")
    try:
        # both sides of each selector threshold (algorithm_selector.cc:107-131: LL8 / LL16 at 16 KiB,
        # LL16 / bulk at 1 MiB) timed on this node, default launch shapes for the LL paths
        cross = {}
        bulk_c = (("fullmesh", 64, 512), ("rsag_zc", 64, 512))
        if ndev_shared(n):
            bulk_c = tuple((a, max(8, 256 // n), 512) for a, _, _ in bulk_c)
        for kb in CROSSOVER_KIB:
            x0, xs = lcg_pair(kb * 512)
            os_ = torch.empty_like(xs)
            cands = (("allpair", 0, 0), ("packet", 0, 0)) if kb <= 64 else (("packet", 0, 0),) + bulk_c
            row = {}
            for a, nb_, nt_ in cands:
                try:
                    if vf:
                        checks[f"crossover:{kb}KiB:{a}:{nb_}x{nt_}"] = vf["check_run"](a, nb_, nt_, kb << 10,
                                                                                      bufs=(x0, xs, os_))
                    for _ in range(3):
                        comm.all_reduce(xs, os_, algo=a, nblocks=nb_, nthreads=nt_)
                    torch.cuda.synchronize()
                    barrier()
                    row[f"{a}:{nb_}x{nt_}"] = round(tmax(_time_calls(
                        lambda: comm.all_reduce(xs, os_, algo=a, nblocks=nb_, nthreads=nt_), 20)) * 1e6, 2)
                except Exception as e:  # noqa: BLE001
                    row[f"{a}:{nb_}x{nt_}"] = str(e)[:80]
            best = min((v, k) for k, v in row.items() if isinstance(v, float))
            # within 3 % the built-in selector's choice stands (timing noise must not flip a threshold)
            sel = SELECT_NAMES[m.lib().mscclppAmdSelectAlgo(n, kb << 10, 0)]
            keep = [k for k, v in row.items() if k.startswith(sel + ":") and isinstance(v, float) and v <= 1.03 * best[0]]
            cross[f"{kb}KiB"] = {"us": row, "best": keep[0] if keep else best[1]}
            del x0, xs, os_
        extras["selector_crossover"] = cross
    except Exception as e:
        extras["selector_crossover_error"] = str(e)[-300:]
    progress("extras: ReduceScatter / AllGather")
    try:
        # ncclReduceScatter / ncclAllGather (row f2) at the headline bucket: 48 MiB of fp16 in per rank
        # for the reduce-scatter, its 48/n MiB result gathered back; both checked bit-exactly (the
        # reduce-scatter in the fullmesh order own-then-ascending, the gather byte for byte)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib as O

        blk = (args.bytes // n) // 16 * 16
        x = lcg_tensor(blk * n // 2, comm.rank, 2, torch.float16, dev)
        rs = torch.empty(blk // 2, dtype=torch.float16, device=dev)
        ag = torch.empty(blk * n // 2, dtype=torch.float16, device=dev)
        for _ in range(2):
            comm.reduce_scatter(x, rs)
            comm.all_gather(rs, ag)
        torch.cuda.synchronize()
        bw = blk // 4
        ins = [O.lcg(O.F16, blk * n // 2, r, 2) for r in range(n)]
        full = O.allreduce_owned(O.F16, O.SUM, [a.view(np.uint32) for a in ins], bw * n, bw * n, bw, 0)[: bw * n]
        mine = full[comm.rank * bw:(comm.rank + 1) * bw]
        ok_rs = bool(np.array_equal(rs.view(torch.uint8).cpu().numpy().view(np.uint32), mine))
        ok_ag = bool(np.array_equal(ag.view(torch.uint8).cpu().numpy().view(np.uint32), full))
        # every rank computed the oracle above at its own pace: line the ranks up before each timed
        # loop, or the first call of a fast rank waits in its handshake for a slow one (round 3's
        # rehearsal lines timed 1.2-10 ms of reduce-scatter that way; the kernel takes ~120 us)
        torch.cuda.synchronize()
        barrier()
        t_rs = tmax(_time_calls(lambda: comm.reduce_scatter(x, rs), 5))
        barrier()
        t_ag = tmax(_time_calls(lambda: comm.all_gather(rs, ag), 5))
        extras["reduce_scatter_allgather"] = {
            "bytes_in_per_rank_rs": blk * n, "bytes_out_per_rank_ag": blk * n,
            "reduce_scatter_us": round(t_rs * 1e6, 1), "all_gather_us": round(t_ag * 1e6, 1),
            # nccl-tests convention: algbw = total buffer bytes / t (recvcount * n for both)
            "reduce_scatter_algbw_GBs": round(blk * n / t_rs / 1e9, 1),
            "all_gather_algbw_GBs": round(blk * n / t_ag / 1e9, 1),
            # every rank's check (a max over ranks of "differs")
            "correct_bitexact": {"reduce_scatter": tmax(0.0 if ok_rs else 1.0) == 0.0,
                                 "all_gather": tmax(0.0 if ok_ag else 1.0) == 0.0}}
        checks.update(extras["reduce_scatter_allgather"]["correct_bitexact"])
        del x, rs, ag
    except Exception as e:
        extras["reduce_scatter_allgather_error"] = str(e)[-300:]
    progress("extras: fp32 1 GiB ring-order RS+AG")
    try:
        # BASELINE configs[4]: both ring-order kernels (the same order-stable sum, own then r+1, ...):
        # through the 128 MiB bulk scratch in several passes (rsag) and zero-copy (rsag_zc)
        # Inputs: ring_tensor (random signs, 8 exponents, full mantissas), so that the 0-ulp check
        # below tells the ring order from any other; every rank checks its whole output against the
        # ring-order sum computed on its own device, and a sample against the CPU oracle
        S = 1 << 30
        count = S // 4
        x0, x1 = (ring_tensor(0, count, rank, sq, dev) for sq in (0, 1))
        os_ = torch.empty_like(x0)
        peak = n * XGMI_LINK_GBS / 2
        for a in ("rsag", "rsag_zc"):
            row = {}
            if vf:
                comm.all_reduce(x0, os_, algo=a)
                vf["poison"](os_)
                comm.all_reduce(x1, os_, algo=a)
                torch.cuda.synchronize()
                bad = ring_order_mismatches(os_, n, 1)
                sample = ring_oracle_sample(os_, n, 1)
                row["mismatched_elements_max_over_ranks"] = int(tmax(float(bad)))
                row["oracle_sample_ok"] = vf["all_ok"](sample)
                checks[f"fp32_1GiB_{a}"] = vf["all_ok"](bad == 0 and sample and comm.device_error() == 0)
            for _ in range(2):
                comm.all_reduce(x1, os_, algo=a)
            torch.cuda.synchronize()
            barrier()
            t = tmax(_time_calls(lambda: comm.all_reduce(x1, os_, algo=a), 5))
            ach = S / t / 1e9
            row.update({"ms": round(t * 1e3, 3), "algbw_GBs": round(ach, 2),
                        "busbw_GBs": round(ach * 2 * (n - 1) / n, 2), "peak": round(peak, 1),
                        "frac": round(ach / peak, 4),
                        "peak_source": "n * 153.6 / 2 GB/s, the all-pairs AllReduce algbw ceiling (BASELINE.md §2)",
                        # SURVEY §8(d) config 5's contrast: one ring over one link per hop moves
                        # 2(n-1)/n * S through each link, algbw <= 153.6 * n / (2(n-1)) GB/s
                        "ring_one_link_bound": round(XGMI_LINK_GBS * n / (2 * (n - 1)), 1)})
            extras[f"fp32_1GiB_{a}"] = row
        del x0, x1, os_
    except Exception as e:
        extras["fp32_1GiB_error"] = str(e)[-300:]
    progress("extras: graph-captured LL latency sweep")
    try:
        glat = {}
        # the first graph a process times runs slow (a one-time cost, tools/ll_small_probe.py:
        # 32 us for the first size, 3.3 us for the same size measured again) -- discard one
        xw = torch.rand(512, device=dev).half()
        graph_time_per_call(lambda: comm.all_reduce(xw, torch.empty_like(xw)), sync=barrier)
        for kb in LL_SWEEP_KIB:
            a0, a1 = lcg_pair(kb * 512)
            os_ = torch.empty_like(a0)
            t, g = graph_time_per_call(lambda: comm.all_reduce(a0, os_), sync=barrier, keep=True)
            glat[f"{kb}KiB"] = round(tmax(t) * 1e6, 2)
            if vf:  # the captured calls on new data: the replay must produce the seq-1 result
                checks[f"ll_graph:{kb}KiB"] = vf["check_replay"](g, a0, a1, os_, kb << 10)
            del g
        extras["ll_latency_graph_us"] = glat
    except Exception as e:
        extras["ll_latency_graph_error"] = str(e)[-300:]
    progress("extras: mscclpp-test kernels")
    try:
        # the mscclpp-test kernels on the sizes the reference publishes (BASELINE.md §1,
        # test/deploy/perf_ndmv4.jsonl / perf_ndmv5.jsonl), timed like common.cc:202-227
        # (20 calls in one graph, 15 launches), int32 data = rank
        mt = {}
        for k, kb, pub in (("k2", 8, "A100 6.51 us (8 ranks, perf_ndmv4.jsonl:5)"),
                           ("k6", 24, "A100 7.24 us / H100 6.18 us"), ("k6", 48, "A100 7.91 us / H100 6.62 us"),
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
            if k != "k5":  # out of place: every element is 0 + 1 + ... + (n-1) after the replays
                torch.cuda.synchronize()
                good = bool(torch.all(os_ == n * (n - 1) // 2).item()) and comm.device_error() == 0
                row["correct"] = vf["all_ok"](good) if vf else good
                checks[f"{k}_{kb}KiB"] = row["correct"]
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
        checks["k1_1GiB"] = vf["all_ok"](ok) if vf else bool(ok)
        extras["mscclpp_test"] = mt
    except Exception as e:
        extras["mscclpp_test_error"] = str(e)
    extras["device_error"] = comm.device_error()
    return extras


def launch_ranks(n, args):
    """`bench.py --gpus N` without WORLD_SIZE: start N rank processes of this script with the
    torch.distributed.run environment (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*).  This parent never
    touches the GPU; rank 0 prints the JSON line.  Returns the exit code (first failing rank's)."""
    import signal
    import socket
    import subprocess

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      start_new_session=True))
    deadline = time.time() + args.rank_timeout
    rc = 0
    while procs and any(p.poll() is None for p in procs):
        failed = [p for p in procs if p.returncode not in (None, 0)]
        if failed or time.time() > deadline:
            rc = failed[0].returncode if failed else 124
            print(f"bench launcher: {'rank exited with ' + str(rc) if failed else 'timeout'}; stopping the ranks",
                  file=sys.stderr, flush=True)
            time.sleep(20 if failed else 0)  # let peers report their own error first
            for p in procs:
                if p.poll() is None:
                    os.killpg(p.pid, signal.SIGTERM)
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    os.killpg(p.pid, signal.SIGKILL)
            break
        time.sleep(0.2)
    for p in procs:
        p.wait()
        if rc == 0 and p.returncode:
            rc = p.returncode
    return rc


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        n = args.gpus or 1
        if n > 1:
            sys.exit(launch_ranks(n, args))
        world = 1
    else:
        world = int(env_world)
        if args.gpus is not None and args.gpus != world:
            print(f"bench: --gpus {args.gpus} disagrees with WORLD_SIZE={world}", file=sys.stderr)
            sys.exit(2)
    if args.dry_run:  # no GPU touched: the launcher / environment contract only
        rank = int(os.environ.get("RANK", "0"))
        assert 0 <= rank < world and int(os.environ.get("LOCAL_RANK", rank)) == rank
        if os.environ.get("BENCH_DRY_RUN_FAIL_RANK") == str(rank):
            sys.exit(3)
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": world, "master": os.environ.get("MASTER_ADDR"),
                              "port": os.environ.get("MASTER_PORT")}), flush=True)
        return
    res = bench_multi(args) if world > 1 else bench_single(args)
    if res is not None:
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
