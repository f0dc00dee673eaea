"""Phase breakdown (PhaseTrace) of the LL kernels with 8 ranks in one launch on one GPU."""
import json, os, sys
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import mscclpp_amd as m
N = 8
torch.cuda.set_device(0)
res = {}
for name, count in (("allpair", 512), ("allpair", 8192), ("packet", 512), ("packet", 1 << 19)):
    a = m.ALGO_NAMES[name]
    sb = m.scratch_required(a, N, count * 2, m.F16)
    ranks = m.InProcessRanks(N, sb)
    ins = [torch.rand(count, device="cuda").half() for _ in range(N)]
    outs = [torch.empty_like(x) for x in ins]
    for _ in range(5):
        ranks.all_reduce(ins, outs, a)
    torch.cuda.synchronize()
    with m.PhaseTrace() as tr:
        for _ in range(4):
            ranks.all_reduce(ins, outs, a)
    res[f"{name}:{count*2>>10}KiB"] = {v: tr.phases(name, v) for v in (0, 7)}
print(json.dumps(res, indent=1))
