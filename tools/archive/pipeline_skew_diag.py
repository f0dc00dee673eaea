"""Diagnostic: rsag_pipeline captured in a graph, replayed with new data under rank skew."""
import multiprocessing as mp, os, sys, time, traceback
import numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", ".")); sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "tests"))

def worker(rank, n, uid, q, mode):
    try:
        os.environ.setdefault("MSCCLPP_AMD_SPIN_TIMEOUT_MS", "5000")
        import torch, mscclpp_amd as m, oracle_lib as O
        torch.cuda.set_device(0)
        comm = m.Communicator(rank, n, uid)
        count = 1 << 18
        x = torch.zeros(count, dtype=torch.float32, device="cuda"); y = torch.zeros_like(x)
        comm.all_reduce(x, y, algo="rsag_pipeline"); torch.cuda.synchronize()
        if mode == "graph":
            side = torch.cuda.Stream(); side.wait_stream(torch.cuda.current_stream())
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=side):
                comm.all_reduce(x, y, algo="rsag_pipeline")
            torch.cuda.synchronize()
        res = []
        prev = None
        for k in range(12):
            ins = [O.lcg(2, count, r, 40 + k) for r in range(n)]
            x.copy_(torch.from_numpy(ins[rank].view(np.int32).copy()).view(torch.float32))
            y.fill_(-1)
            torch.cuda.synchronize()
            if rank == 1 and k % 2: time.sleep(0.05)  # skew: rank 1 late every other call
            if mode == "graph": g.replay()
            else: comm.all_reduce(x, y, algo="rsag_pipeline")
            torch.cuda.synchronize()
            got = y.cpu().numpy()
            ref = (ins[0].view(np.float32).astype(np.float64) + ins[1].view(np.float32).astype(np.float64))
            bad = np.nonzero(~np.isclose(got, ref, rtol=1e-5, atol=1e-5))[0]
            info = (k, int(bad.size))
            if bad.size:
                stale = int(np.isclose(got[bad], prev[bad], rtol=1e-5, atol=1e-5).sum()) if prev is not None else -1
                info += (int(bad[0]), int(bad[-1]), int((got[bad] == -1).sum()), stale)
            res.append(info)
            prev = ref
        res.append(("err", comm.device_error()))
        comm.barrier(); comm.destroy()
        q.put((rank, res, None))
    except Exception:
        q.put((rank, None, traceback.format_exc()))

if __name__ == "__main__":
    import mscclpp_amd as m
    for mode in ("eager", "graph"):
        uid = m.Communicator.unique_id()
        ctx = mp.get_context("spawn"); q = ctx.Queue()
        ps = [ctx.Process(target=worker, args=(r, 2, uid, q, mode)) for r in range(2)]
        [p.start() for p in ps]
        for _ in range(2):
            print(mode, q.get(timeout=200), flush=True)
        [p.join(30) for p in ps]
