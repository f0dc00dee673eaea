"""Phase breakdown (PhaseTrace) of the bulk kernels with 8 ranks in one launch on one GPU, 48 MiB fp16
per rank: where a fabric-free call spends its time (handshake waits vs data movement)."""
import json, os, sys
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import mscclpp_amd as m
N, S = 8, 48 << 20
count = S // 2
torch.cuda.set_device(0)
ins = [torch.rand(count, device="cuda").half() for _ in range(N)]
outs = [torch.empty_like(a) for a in ins]
ranks = m.InProcessRanks(N, 1 << 20, bulk_scratch_bytes=S + (16 << 20))
res = {}
for name, nb, nt in (("rsag_zc", 32, 512), ("fullmesh", 32, 512), ("rsag_zc", 16, 512), ("fullmesh", 64, 256)):
    a = m.ALGO_NAMES[name]
    for _ in range(3):
        ranks.all_reduce(ins, outs, a, nblocks=nb, nthreads=nt)
    torch.cuda.synchronize()
    with m.PhaseTrace() as tr:
        for _ in range(4):
            ranks.all_reduce(ins, outs, a, nblocks=nb, nthreads=nt)
    res[f"{name}:{nb}x{nt}"] = {f"view{v}": tr.phases(name, v) for v in (0, 7)}
print(json.dumps(res, indent=1))
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open("gpurun_out/trace_probe.json", "w"), indent=1)
