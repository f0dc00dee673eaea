"""Workload for a rocprofv3 --pmc pass over the multi-rank kernels (8 ranks in one launch on one GPU,
48 MiB fp16 per rank for the bulk kernels, 1 MiB for LL16): ALGOS (comma list) x 5 calls each.
tools/pmc_multirank.sh runs it under FETCH_SIZE and WRITE_SIZE passes and compares with the
algorithmic bytes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mscclpp_amd as m  # noqa: E402

N = 8
torch.cuda.set_device(0)
for spec in os.environ.get("ALGOS", "rsag_zc:32x512,fullmesh:32x512,packet:0x0").split(","):
    name, shape = spec.split(":")
    nb, nt = (int(v) for v in shape.split("x"))
    S = (1 << 20) if name in ("packet", "allpair") else (48 << 20)
    ins = [torch.rand(S // 2, device="cuda").half() for _ in range(N)]
    outs = [torch.empty_like(a) for a in ins]
    sb = m.scratch_required(m.ALGO_PACKET, N, S, m.F16) if name == "packet" else 1 << 20
    ranks = m.InProcessRanks(N, sb, bulk_scratch_bytes=S + (16 << 20))
    for _ in range(5):
        ranks.all_reduce(ins, outs, m.ALGO_NAMES[name], nblocks=nb, nthreads=nt)
    torch.cuda.synchronize()
    assert ranks.errors() == [0] * N
    del ranks, ins, outs
    torch.cuda.empty_cache()
print("pmc workload done")
