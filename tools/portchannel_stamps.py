"""Where a PortChannel iteration's time goes: the 2-rank all-to-all
at 1 MiB per peer (mscclppAmdPortChannelAllToAllStats with the proxy's trigger stamps), for each
token-update mechanism (MSCCLPP_AMD_TOKEN_WRITE = memcpy | writevalue) in fresh rank processes, and
the reference tutorial's bidirectional putWithSignal (tests/bin/test_reference_setup port) under each.

Prints one JSON object per (mechanism, mode) and per tutorial run.  Run on the GPU box."""
import ctypes
import json
import multiprocessing as mp
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = ["put+signal", "putWithSignal", "putWithSignalAndFlush"]
KEYS = ["us_wall_mean", "correct", "numa", "median", "min", "max", "slowest", "max_poll_gap",
        "launch_to_data_done", "launch_to_token_done", "token_done_to_end", "host_submit_data",
        "host_submit_token", "host_handler", "slowest_launch_to_token_done", "stamps"]


def worker(rank, uid, iters, q):
    try:
        import torch

        import mscclpp_amd as m

        torch.cuda.set_device(0)
        L = m.lib()
        L.mscclppAmdPortChannelAllToAllStats.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                                         ctypes.POINTER(ctypes.c_double), ctypes.c_int]
        comm = m.Communicator(rank, 2, uid)
        res = {}
        for mode in (0, 1, 2):
            o = (ctypes.c_double * 16)()
            m.check(L.mscclppAmdPortChannelAllToAllStats(comm.comm, 1 << 20, mode, iters, o, 16), "stats")
            res[NAMES[mode]] = {k: round(o[i], 2) for i, k in enumerate(KEYS)}
        comm.destroy()
        q.put((rank, res, None))
    except Exception:  # noqa: BLE001
        import traceback

        q.put((rank, None, traceback.format_exc()))


def run(token, iters=200, priority=""):
    import mscclpp_amd as m

    os.environ["MSCCLPP_AMD_TOKEN_WRITE"] = token
    os.environ["MSCCLPP_AMD_COPY_STREAM_PRIORITY"] = priority
    os.environ["MSCCLPP_AMD_PROXY_GAP_STATS"] = "1"
    uid = m.Communicator.unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, uid, iters, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = {}
    try:
        for _ in range(2):
            rank, res, err = q.get(timeout=120)
            if err:
                raise RuntimeError(err)
            got[rank] = res
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return got


def tutorial(token):
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MSCCLPP_AMD_TOKEN_WRITE=token)
    r = subprocess.run([os.path.join(ROOT, "tests", "bin", "test_reference_setup"), "port", str(port)],
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=120, env=env)
    rows = [json.loads(x.split(" ", 1)[1]) for x in r.stdout.splitlines() if x.startswith("PORT_JSON ")]
    return {"rc": r.returncode, "rows": rows, "tail": r.stdout[-300:] if r.returncode else ""}


def summary(rec):
    """Median over both ranks of each column, per mode."""
    out = {}
    for mode in NAMES:
        rows = [r[mode] for r in rec.values()]
        out[mode] = {k: round(sorted(x[k] for x in rows)[len(rows) // 2], 2) for k in KEYS[3:]}
    return out


if __name__ == "__main__":
    tokens = sys.argv[1].split(",") if len(sys.argv) > 1 else ["memcpy", "writevalue"]
    prios = sys.argv[2].split(",") if len(sys.argv) > 2 else [""]
    for tok in tokens:
        for prio in prios:
            print(json.dumps({"token_write": tok, "copy_stream_priority": prio or "normal",
                              "tutorial": tutorial(tok) if not prio else None}), flush=True)
            rec = run(tok, priority=prio)
            print(json.dumps({"token_write": tok, "copy_stream_priority": prio or "normal",
                              "alltoall_1MiB": rec, "summary": summary(rec)}), flush=True)
