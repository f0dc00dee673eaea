"""BASELINE config 1: the host-proxy path of test/allgather_test_host_offloading.cu (2 ranks,
4 KiB, CPU proxy thread per rank moves the bytes with hipMemcpyAsync), run on this library.

Prints one JSON object: us per kernel without / with graph, algbw, correctness, cores used.
Ranks are processes (spawn); on a 1-GPU box both use cuda:0 (loopback), as the config describes."""
import ctypes
import json
import multiprocessing as mp
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


PINGPONG_ITERS = 100000  # timed MemoryChannel ping-pong iterations (>= 100k)
PC_ITERS = 20  # PortChannel all-to-all iterations per mode (median / min / max over >= 20)


def worker(rank, n, uid, size, q):
    try:
        import torch

        import mscclpp_amd as m

        ndev = torch.cuda.device_count()
        torch.cuda.set_device(rank % ndev)
        L = m.lib()
        L.mscclppAmdHostOffloadAllGather.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                                     ctypes.POINTER(ctypes.c_double)]
        L.mscclppAmdPortChannelAllToAllStats.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                                         ctypes.POINTER(ctypes.c_double), ctypes.c_int]
        comm = m.Communicator(rank, n, uid)
        out = (ctypes.c_double * 4)()
        print(f"[host_proxy rank {rank}/{n}] host-offload loop", file=sys.stderr, flush=True)
        m.check(L.mscclppAmdHostOffloadAllGather(comm.comm, size, 10, 10, out), "host offload")
        print(f"[host_proxy rank {rank}/{n}] PortChannel all-to-all", file=sys.stderr, flush=True)
        res = {"us_per_kernel_nograph": out[0], "us_per_kernel_graph": out[1], "correct": out[2] == 1.0,
               "proxy_numa_node": int(out[3]), "device": rank % ndev}
        pc = {}
        for mode in (0, 1, 2):
            # PC_ITERS back-to-back iterations after one untimed launch; each iteration's own time from
            # HIP events: median (the row's figure), min and max, and the slowest iteration's index
            o = (ctypes.c_double * 8)()
            m.check(L.mscclppAmdPortChannelAllToAllStats(comm.comm, 1 << 20, mode, PC_ITERS, o, 8), "portchannel")
            pc[["put+signal", "putWithSignal", "putWithSignalAndFlush"][mode]] = {
                "us": round(o[3], 2), "min_us": round(o[4], 2), "max_us": round(o[5], 2),
                "mean_us_wall": round(o[0], 2), "slowest_iteration": int(o[6]), "iterations": PC_ITERS,
                "proxy_max_poll_gap_us": round(o[7], 1), "correct": o[1] == 1.0}
        res["portchannel_alltoall_1MiB"] = pc
        if n == 2:
            # the reference's MemoryChannel packet ping-pong latency (memory_channel_tests.cu:98-107):
            # 1024 ints, PINGPONG_ITERS one-way hand-offs per packet type after 1000 checked ones
            L.mscclppAmdMemChannelPingPong.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                       ctypes.POINTER(ctypes.c_double), ctypes.c_int]
            pp = {}
            for name, ll8 in (("ll16", 0), ("ll8", 1)):
                print(f"[host_proxy rank {rank}/{n}] {name} ping-pong", file=sys.stderr, flush=True)
                o = (ctypes.c_double * 6)()
                m.check(L.mscclppAmdMemChannelPingPong(comm.comm, 1024, PINGPONG_ITERS, ll8, o, 6), "ping-pong")
                pp[name] = {"us_per_iter": round(o[0], 3), "correct": o[1] == 1.0,
                            "error_record": [int(o[k]) for k in range(2, 6)]}
            res["pingpong"] = pp
        comm.destroy()
        q.put((rank, res, None))
    except Exception as e:  # noqa: BLE001
        import traceback

        q.put((rank, None, traceback.format_exc()))


def run(n=2, size=4096, timeout=180):
    import mscclpp_amd as m

    # every proxy thread records its longest gap between FIFO polls (a clock read per poll): a gap
    # near an iteration's stall says the thread was off the CPU (host side), DESIGN.md §9
    saved = os.environ.get("MSCCLPP_AMD_PROXY_GAP_STATS")
    os.environ.setdefault("MSCCLPP_AMD_PROXY_GAP_STATS", "1")  # inherited by the spawned ranks only
    uid = m.Communicator.unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, n, uid, size, q)) for r in range(n)]
    for p in ps:
        p.start()
    if saved is None:
        del os.environ["MSCCLPP_AMD_PROXY_GAP_STATS"]
    got = {}
    deadline = time.monotonic() + timeout
    try:
        for _ in range(n):
            rank, res, err = q.get(timeout=max(1.0, deadline - time.monotonic()))
            if err:
                raise RuntimeError(err)
            got[rank] = res
    except BaseException:
        for p in ps:  # a rank that failed or stalled: none of its peers may keep spinning on the GPU
            p.kill()
        for p in ps:
            p.join(timeout=30)
        raise
    for p in ps:
        p.join(timeout=30)
    r0 = got[0]
    us = r0["us_per_kernel_graph"]
    return {"value": round(size / (us * 1e-6) / 1e9, 4), "unit": "GB/s", "us_per_kernel_graph": round(us, 2),
            "us_per_kernel_nograph": round(r0["us_per_kernel_nograph"], 2), "bytes": size, "ranks": n,
            "correct": all(g["correct"] for g in got.values()),
            "cores": 2 * n, "cores_note": "per rank: 1 busy-poll proxy thread + 1 launching thread",
            "proxy_numa_node": r0["proxy_numa_node"], "portchannel_alltoall_1MiB": r0["portchannel_alltoall_1MiB"],
            "pingpong": r0.get("pingpong"),
            "devices": sorted({g["device"] for g in got.values()}),
            "pingpong_correct": all(g.get("pingpong", {}).get(k, {}).get("correct", False)
                                    for g in got.values() for k in ("ll16", "ll8")) if n == 2 else None,
            "path": "test/allgather_test_host_offloading.cu restated on libmscclpp_amd (FIFO + proxy + hipMemcpyAsync)"}


if __name__ == "__main__":
    print(json.dumps(run(int(sys.argv[1]) if len(sys.argv) > 1 else 2)), flush=True)
