import sys, os, numpy as np, torch
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import mscclpp_amd as m, oracle_lib as O
for (n, dt, block, nb) in [(8, 2, 12288, 8), (8, 2, 12288, 4), (8, 0, 24576, 8), (4, 2, 12288, 8), (8, 2, 16384, 8), (8, 2, 12288, 6)]:
    item = 2 if dt < 2 else 4
    tdt = {0: torch.float16, 2: torch.float32}[dt]
    count = block * n
    for rep in range(3):
        ranks = m.InProcessRanks(n, 1 << 16, bulk_scratch_bytes=max(count * item, 1 << 20))
        ins = [O.lcg(dt, count, r, 0) for r in range(n)]
        dins = [torch.from_numpy(a.view(np.int16 if item == 2 else np.int32).copy()).view(tdt).cuda() for a in ins]
        douts = [torch.zeros(block, dtype=tdt, device="cuda") for _ in range(n)]
        ranks.collective(1, dins, douts, nblocks=nb, budget_ticks=100_000_000)
        torch.cuda.synchronize()
        print(n, dt, block, nb, rep, "errors", ranks.errors(), flush=True)
