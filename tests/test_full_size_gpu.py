"""Parity at BASELINE.json's full sizes (configs[1], [2], [3] upper end, [4]).

* configs[1]: the 48 MiB fp16 LL16 self-reduce -- output AND the 96 MiB packet image (flag and data
  words) bit-exact against the C oracle, for two consecutive flags.
* configs[2]: 8 ranks x 48 MiB fp16 (2048 x 12288) through the bulk fullmesh and zero-copy RS+AG
  kernels -- every rank's output bit-exact against the oracle in the reference's sum orders.
* configs[3] upper end: 8 ranks x 1 MiB fp16 LL16 two-hop, output and scratch image bit-exact.
* configs[4]: 8 ranks x 1 GiB fp32 RS+AG in ring order (scratch-based and zero-copy): all eight
  outputs identical, EVERY element equal to the ring-order fp32 sum x_o + x_{o+1} + ... (o = the slice
  owner, allreduce_rsag.cu:85-94) computed by torch on the device in the same order, and 1 Mi sampled
  elements plus every slice boundary equal the same sum computed in numpy -- 0 ulp.
All ranks run in one process on one GPU (one launch, blockIdx.y = rank)."""
import numpy as np
import pytest
import torch

import oracle_lib as O

pytestmark = pytest.mark.gpu


def _dev16(a):
    return torch.from_numpy(a.view(np.int16).copy()).view(torch.float16).cuda()


def _u32(t):
    return t.cpu().contiguous().view(torch.uint8).numpy().view(np.uint32)


def test_self_reduce_48MiB_bit_exact(built):
    import mscclpp_amd as m

    nbytes = 48 << 20
    count = nbytes // 2
    x = O.lcg(O.F16, count, 0, 0)
    y = O.lcg(O.F16, count, 1, 0)
    xd, yd = _dev16(x), _dev16(y)
    out = torch.empty_like(xd)
    pk = m.DeviceBuffer(2 * nbytes)
    flags = torch.ones(m.FLAG_SLOTS, dtype=torch.int32, device="cuda")
    err = torch.zeros(16, dtype=torch.int32, device="cuda")
    try:
        for flag in (1, 2):
            out.zero_()
            m.self_reduce_ll16(xd, yd, pk.ptr, out, flags, err)
            torch.cuda.synchronize()
            assert int(err[0].item()) == 0
            pkts, exp = O.self_reduce(O.F16, O.SUM, x, y, flag)
            assert np.array_equal(_u32(out), exp), f"output, flag {flag}"
            img = m.device_view(pk.ptr, 2 * nbytes).cpu().numpy().view(np.uint32)
            assert np.array_equal(img, pkts.view(np.uint32)), f"packet image, flag {flag}"
    finally:
        pk.free()


@pytest.mark.parametrize("algo,order", [("fullmesh", 0), ("rsag_zc", 1)])
def test_allreduce_8x48MiB_fp16_bit_exact(built, algo, order):
    import mscclpp_amd as m

    n, nbytes = 8, 48 << 20
    count = nbytes // 2
    slice_bytes = nbytes // n
    ranks = m.InProcessRanks(n, 1 << 16, bulk_scratch_bytes=n * slice_bytes if algo == "fullmesh" else 0)
    ins = [O.lcg(O.F16, count, r, 0) for r in range(n)]
    dins = [_dev16(a) for a in ins]
    douts = [torch.zeros_like(d) for d in dins]
    for _ in range(2):  # second call re-uses the semaphores and (fullmesh) scratch of the first
        ranks.all_reduce(dins, douts, m.ALGO_NAMES[algo], nblocks=32, nthreads=256)
    torch.cuda.synchronize()
    assert ranks.errors() == [0] * n
    exp = O.allreduce_sliced(O.F16, O.SUM, [a.view(np.uint32) for a in ins], nbytes // 4, slice_bytes // 4, order)
    for r in range(n):
        assert np.array_equal(_u32(douts[r]), exp[r]), f"rank {r}"


def test_ll16_8x1MiB_fp16_bit_exact(built):
    import mscclpp_amd as m

    n, count = 8, 1 << 19
    sb = m.scratch_required(m.ALGO_PACKET, n, count * 2, O.F16)
    ranks = m.InProcessRanks(n, sb)
    for flag in (1, 2, 3):
        ins = [O.lcg(O.F16, count, r, flag) for r in range(n)]
        dins = [_dev16(a) for a in ins]
        douts = [torch.zeros_like(d) for d in dins]
        ranks.all_reduce(dins, douts, m.ALGO_PACKET, nblocks=28, nthreads=512)
        torch.cuda.synchronize()
        assert ranks.errors() == [0] * n
        exp, scr = O.allreduce_packet(O.F16, O.SUM, ins, count, flag, sb // 2)
        for r in range(n):
            assert np.array_equal(_u32(douts[r]), exp[r][: count // 2]), f"rank {r}, flag {flag}"
        if flag == 1:
            for r in range(n):
                assert np.array_equal(ranks.scratch_tensor(r, sb).cpu().numpy().view(np.uint32), scr[r])


@pytest.mark.parametrize("algo", ["rsag", "rsag_zc"])
def test_rsag_ring_8x1GiB_fp32(built, algo):
    """Every one of the 8 x 268 M outputs equals the ring-order fp32 sum x_o + x_{o+1} + ... (o = the
    slice owner, allreduce_rsag.cu:85-94; allreduce_rsag_zero_copy.cu:88-98) computed elementwise by
    torch on the device in the same order (IEEE fp32 adds: 0 ulp), and 1 Mi sampled elements plus
    every slice boundary equal the same sum computed on the CPU in numpy."""
    import mscclpp_amd as m

    n, nbytes = 8, 1 << 30
    count = nbytes // 4
    slice_elems = count // n
    free, _ = torch.cuda.mem_get_info()
    if free < 28 << 30:
        pytest.skip("needs ~26 GiB of device memory")
    ranks = m.InProcessRanks(n, 1 << 16, bulk_scratch_bytes=nbytes if algo == "rsag" else 0)
    g = torch.Generator(device="cuda")
    ins = []
    for r in range(n):
        g.manual_seed(1000 + r)
        ins.append(torch.rand(count, generator=g, device="cuda") * 2 - 1)
    outs = [torch.empty_like(t) for t in ins]
    ranks.all_reduce(ins, outs, m.ALGO_NAMES[algo], nblocks=32, nthreads=512)
    torch.cuda.synchronize()
    assert ranks.errors() == [0] * n
    for r in range(1, n):
        assert torch.equal(outs[r].view(torch.int32), outs[0].view(torch.int32)), f"rank {r} differs from rank 0"
    bad = 0
    for o in range(n):  # every element, in the owner's ring order
        sl = slice(o * slice_elems, (o + 1) * slice_elems if o < n - 1 else count)
        acc = ins[o][sl].clone()
        for k in range(1, n):
            acc += ins[(o + k) % n][sl]
        bad += int((acc.view(torch.int32) != outs[0][sl].view(torch.int32)).sum().item())
        del acc
    assert bad == 0, f"{bad} of {count} elements differ from the ring-order sum"
    rng = np.random.default_rng(5)
    idx = np.concatenate([rng.integers(0, count, 1 << 20),
                          np.array([k * slice_elems + d for k in range(n) for d in (0, 1, slice_elems - 1)])])
    it = torch.from_numpy(idx).cuda()
    xs = np.stack([ins[r][it].cpu().numpy() for r in range(n)])  # [n, m]
    owner = idx // slice_elems
    cols = np.arange(idx.size)
    acc = xs[owner, cols].astype(np.float32)
    for k in range(1, n):
        acc = (acc + xs[(owner + k) % n, cols]).astype(np.float32)
    got = outs[0][it].cpu().numpy()
    assert np.array_equal(got.view(np.uint32), acc.view(np.uint32))
    del ranks, ins, outs
    torch.cuda.empty_cache()
