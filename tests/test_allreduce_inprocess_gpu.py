"""GPU parity of the multi-rank AllReduce kernels, with n ranks of one collective running in one
process on one GPU (one launch, blockIdx.y = rank; every rank has its own scratch, flags,
semaphores).  Outputs and, for the LL paths, the whole scratch image (packet flag + data words)
are compared bit-exactly with the CPU oracle; the bulk paths against the oracle's sliced sums in
the reference's sum orders (fullmesh: own then ascending; rsag: ring order)."""
import numpy as np
import pytest
import torch

import oracle_lib as O

pytestmark = pytest.mark.gpu

TORCH = {O.F16: torch.float16, O.BF16: torch.bfloat16, O.F32: torch.float32, O.I32: torch.int32}
ITEM = {O.F16: 2, O.BF16: 2, O.F32: 4, O.I32: 4}


def _dev(arr, dt):
    t = torch.from_numpy(arr.view(np.int16 if arr.dtype == np.uint16 else np.int32).copy())
    return t.view(TORCH[dt]).cuda()


def _bytes(t):
    return t.cpu().contiguous().view(torch.uint8).numpy()


def _inputs(dt, n, count, seq=0, special=False):
    ins = [O.lcg(dt, count, r, seq) for r in range(n)]
    if special:
        rng = np.random.default_rng(11 + seq)
        bits = 16 if ITEM[dt] == 2 else 32
        for r in range(n):
            m = rng.random(count) < 0.25
            ins[r] = ins[r].copy()
            ins[r][m] = rng.integers(0, 2**bits, m.sum(), dtype=np.uint64).astype(ins[r].dtype)
    return ins


def _cmp(got_bytes, exp_bytes, dt):
    if dt == O.F32:
        g = got_bytes.view(np.uint32)
        e = exp_bytes.view(np.uint32)
        nan = (e & 0x7FFFFFFF) > 0x7F800000
        assert np.array_equal(g[~nan], e[~nan])
        assert np.all((g[nan] & 0x7FFFFFFF) > 0x7F800000)
    else:
        bad = np.nonzero(got_bytes != exp_bytes)[0]
        assert bad.size == 0, f"{bad.size} byte mismatches, first {bad[:8]}"


LL_CASES = [
    # (n, dt, count, special)
    (2, O.F16, 4096, False), (4, O.F16, 8192, True), (8, O.F16, 16384, True), (8, O.BF16, 16384, True),
    (8, O.F32, 8192, False), (8, O.I32, 8192, False), (3, O.F16, 3000, False), (8, O.F16, 1000, False),
    (8, O.F16, 777, False), (5, O.F32, 1001, False), (8, O.F16, 262144, False),
    # LL16 step 3's sentinel (from 8192 units per slice) with a ragged last wave and several passes
    (3, O.F16, 100003, True), (5, O.BF16, 165074, False), (7, O.F32, 114787, False),
]


@pytest.mark.parametrize("algo", ["packet", "allpair"])
@pytest.mark.parametrize("n,dt,count,special", LL_CASES)
def test_ll_allreduce_bit_exact(built, algo, n, dt, count, special):
    import mscclpp_amd as m

    algo_code = m.ALGO_PACKET if algo == "packet" else m.ALGO_ALLPAIR
    nbytes = count * ITEM[dt]
    if algo == "allpair" and nbytes > (256 << 10):
        pytest.skip("one-hop LL8 is the <=16 KiB path; keep its scratch small")
    sb = max(m.scratch_required(algo_code, n, nbytes, dt), 1 << 16)
    ranks = m.InProcessRanks(n, sb)
    nblocks = (n - 1) * 2 if algo == "packet" else 4
    for call, flag in enumerate((1, 2, 3)):
        ins = _inputs(dt, n, count, seq=call, special=special)
        dins = [_dev(a, dt) for a in ins]
        douts = [torch.full_like(d, 0) for d in dins]
        ranks.all_reduce(dins, douts, algo_code, nblocks=nblocks, nthreads=256)
        torch.cuda.synchronize()
        assert ranks.errors() == [0] * n
        if algo == "packet":
            exp, scr = O.allreduce_packet(dt, O.SUM, ins, count, flag, sb // 2)
        else:
            exp, scr = O.allreduce_allpairs(dt, O.SUM, ins, count, flag, sb // 2)
        for r in range(n):
            _cmp(_bytes(douts[r]), exp[r].view(np.uint8)[:nbytes], dt)
        if call == 0:
            # packet image of the flag-1 half: flag words and data words, bit-exact
            for r in range(n):
                got = ranks.scratch_tensor(r, sb).cpu().numpy().view(np.uint32)
                assert np.array_equal(got, scr[r]), f"scratch image of rank {r}"


@pytest.mark.parametrize("count", [262144, 524288, 262146, 262147, 1023])
def test_ll8_two_ranks_default_shape_bit_exact(built, count):
    """at 2 ranks the selector sends the whole LL range (to 1 MiB) to one-hop LL8 with its
    default grid (nblocks = nthreads = 0: up to 128 x 512 lanes, poll_units / waveSingle).  Outputs
    and the flag-1 scratch image bit-exact at 512 KiB, 1 MiB, an odd LL8 word count (a trailing
    single packet), a ragged tail below one word, and a small bucket, over three flags."""
    import mscclpp_amd as m

    n, dt = 2, O.F16
    nbytes = count * 2
    assert m.lib().mscclppAmdSelectAlgo(n, nbytes, dt) == m.ALGO_ALLPAIR
    sb = max(m.scratch_required(m.ALGO_ALLPAIR, n, nbytes, dt), 1 << 16)
    ranks = m.InProcessRanks(n, sb)
    for call, flag in enumerate((1, 2, 3)):
        ins = _inputs(dt, n, count, seq=call, special=(call == 1))
        dins = [_dev(a, dt) for a in ins]
        douts = [torch.full_like(d, 0) for d in dins]
        ranks.all_reduce(dins, douts, m.ALGO_ALLPAIR, nblocks=0, nthreads=0)
        torch.cuda.synchronize()
        assert ranks.errors() == [0] * n
        exp, scr = O.allreduce_allpairs(dt, O.SUM, ins, count, flag, sb // 2)
        for r in range(n):
            _cmp(_bytes(douts[r]), exp[r].view(np.uint8)[:nbytes], dt)
        if call == 0:
            for r in range(n):
                got = ranks.scratch_tensor(r, sb).cpu().numpy().view(np.uint32)
                assert np.array_equal(got, scr[r]), f"scratch image of rank {r}"


@pytest.mark.parametrize("algo,order", [("fullmesh", 0), ("rsag", 1), ("rsag_zc", 1)])
@pytest.mark.parametrize("n,dt,count", [(2, O.F16, 1 << 16), (8, O.F16, 1 << 18), (8, O.F32, 100000),
                                        (4, O.BF16, 65536 + 8), (8, O.I32, 4096), (7, O.F32, 12345),
                                        (8, O.F16, 1001)])
def test_bulk_allreduce_bit_exact(built, algo, order, n, dt, count):
    import mscclpp_amd as m

    algo_code = m.ALGO_NAMES[algo]
    nbytes = count * ITEM[dt]
    slice_bytes = ((nbytes + n - 1) // n + 15) // 16 * 16
    ranks = m.InProcessRanks(n, 1 << 16, bulk_scratch_bytes=max(n * slice_bytes, 1 << 20))
    for call in range(3):
        ins = _inputs(dt, n, count, seq=call, special=(call == 1 and dt != O.F32))
        dins = [_dev(a, dt) for a in ins]
        douts = [torch.full_like(d, 0) for d in dins]
        ranks.all_reduce(dins, douts, algo_code, nblocks=8, nthreads=256)
        torch.cuda.synchronize()
        assert ranks.errors() == [0] * n
        nwords = (nbytes + 3) // 4
        padded = []
        for a in ins:
            w = np.zeros(nwords, np.uint32)
            w.view(np.uint8)[:nbytes] = a.view(np.uint8)
            padded.append(w)
        exp = O.allreduce_sliced(dt, O.SUM, padded, nwords, slice_bytes // 4, order)
        for r in range(n):
            _cmp(_bytes(douts[r]), exp[r].view(np.uint8)[:nbytes], dt)


@pytest.mark.parametrize("algo", ["packet", "allpair", "fullmesh", "rsag_zc"])
def test_in_place(built, algo):
    import mscclpp_amd as m

    n, dt, count = 8, O.F16, 8192
    code = m.ALGO_NAMES[algo]
    nbytes = count * 2
    ranks = m.InProcessRanks(n, max(m.scratch_required(code, n, nbytes, dt), 1 << 16), bulk_scratch_bytes=1 << 20)
    ins = _inputs(dt, n, count)
    bufs = [_dev(a, dt) for a in ins]
    ranks.all_reduce(bufs, bufs, code, nblocks=(n - 1) * 2 if code == m.ALGO_PACKET else 8, nthreads=256)
    torch.cuda.synchronize()
    assert ranks.errors() == [0] * n
    if code in (m.ALGO_FULLMESH, m.ALGO_RSAG_ZC):
        sl = ((nbytes + n - 1) // n + 15) // 16 * 16
        exp = O.allreduce_sliced(dt, O.SUM, [a.view(np.uint32) for a in ins], nbytes // 4, sl // 4,
                                 0 if code == m.ALGO_FULLMESH else 1)
    elif code == m.ALGO_PACKET:
        exp, _ = O.allreduce_packet(dt, O.SUM, ins, count, 1, 1 << 20)
    else:
        exp, _ = O.allreduce_allpairs(dt, O.SUM, ins, count, 1, 1 << 20)
    for r in range(n):
        _cmp(_bytes(bufs[r]), exp[r].view(np.uint8)[:nbytes], dt)


def test_int32_kat(built):
    """mscclpp-test KAT (allreduce_test.cu:1172-1183): input = rank -> n(n-1)/2 everywhere."""
    import mscclpp_amd as m

    n = 8
    for code, nb in ((m.ALGO_ALLPAIR, 4), (m.ALGO_PACKET, 14), (m.ALGO_FULLMESH, 8), (m.ALGO_RSAG, 8),
                     (m.ALGO_RSAG_ZC, 8)):
        count = 1 << 14
        ranks = m.InProcessRanks(n, max(m.scratch_required(code, n, count * 4, O.I32), 1 << 16),
                                 bulk_scratch_bytes=1 << 20)
        ins = [torch.full((count,), r, dtype=torch.int32, device="cuda") for r in range(n)]
        outs = [torch.empty_like(t) for t in ins]
        ranks.all_reduce(ins, outs, code, nblocks=nb, nthreads=256)
        torch.cuda.synchronize()
        assert ranks.errors() == [0] * n
        for o in outs:
            assert torch.all(o == n * (n - 1) // 2)


@pytest.mark.parametrize("n,dt,block", [(2, O.F16, 4096), (8, O.F16, 65536), (8, O.F32, 12288), (4, O.BF16, 2048),
                                        (8, O.I32, 1024)])
def test_reduce_scatter_and_all_gather(built, n, dt, block):
    """ncclReduceScatter / ncclAllGather halves of the bulk path (nccl.cc:662-772), in-process ranks."""
    import mscclpp_amd as m

    item = ITEM[dt]
    count = block * n
    ranks = m.InProcessRanks(n, 1 << 16, bulk_scratch_bytes=max(count * item, 1 << 20))
    for call in range(2):
        ins = _inputs(dt, n, count, seq=call)
        dins = [_dev(a, dt) for a in ins]
        douts = [torch.zeros(block, dtype=TORCH[dt], device="cuda") for _ in range(n)]
        torch.cuda.synchronize()
        pre = [int(e.abs().max().item()) for e in ranks.expected]
        ranks.collective(1, dins, douts)
        torch.cuda.synchronize()
        assert ranks.errors() == [0] * n, ("reduce-scatter", call, pre, ranks.error_details(),
                                           [int(e.abs().max().item()) for e in ranks.expected])
        nw = count * item // 4
        exp = O.allreduce_sliced(dt, O.SUM, [a.view(np.uint32) for a in ins], nw, nw // n, 0)[0]
        for r in range(n):
            _cmp(_bytes(douts[r]), exp.view(np.uint8)[r * block * item:(r + 1) * block * item], dt)
        # all-gather of the reduced blocks reconstructs the AllReduce result on every rank
        gathered = [torch.zeros(count, dtype=TORCH[dt], device="cuda") for _ in range(n)]
        ranks.collective(2, douts, gathered)
        torch.cuda.synchronize()
        assert ranks.errors() == [0] * n, ("all-gather", call, ranks.error_details())
        for r in range(n):
            _cmp(_bytes(gathered[r]), exp.view(np.uint8)[: count * item], dt)


@pytest.mark.parametrize("algo", ["packet", "allpair", "fullmesh", "rsag_zc"])
@pytest.mark.parametrize("dt,count", [(O.I32, 1), (O.F16, 1), (O.F16, 3), (O.F32, 1), (O.BF16, 2), (O.I32, 5)])
@pytest.mark.parametrize("op", [O.SUM, O.MIN])
def test_tiny_buffers(built, algo, dt, count, op):
    """1-5 element buffers (a framework's 4-byte flag all_reduce): every path, SUM and MIN."""
    import mscclpp_amd as m

    n = 2
    code = m.ALGO_NAMES[algo]
    nbytes = count * ITEM[dt]
    ranks = m.InProcessRanks(n, max(m.scratch_required(code, n, nbytes, dt), 1 << 16), bulk_scratch_bytes=1 << 20)
    for call in range(2):
        ins = _inputs(dt, n, count, seq=call)
        dins = [_dev(a, dt) for a in ins]
        douts = [torch.full_like(d, 0) for d in dins]
        try:
            ranks.all_reduce(dins, douts, code, op=op, nblocks=2 if code in (m.ALGO_PACKET, m.ALGO_ALLPAIR) else 2,
                             nthreads=256)
        except RuntimeError as e:  # a path may refuse a size it cannot carry; it must not compute garbage
            pytest.skip(f"{algo} refuses {nbytes} bytes: {e}")
        torch.cuda.synchronize()
        assert ranks.errors() == [0] * n
        exp = O.reduce_seq(dt, op, [np.concatenate([a.view(np.uint8), np.zeros(4, np.uint8)])[: (nbytes + 3) // 4 * 4]
                                    for a in ins])
        for r in range(n):
            _cmp(_bytes(douts[r]), exp.view(np.uint8)[:nbytes], dt)


def _pipeline_expected(dt, op, ins, nbytes, n, R, T):
    """Oracle for allreduceRsAgPipeline (allreduce_rsag_pipeline.cu:85-222): 16-byte unit u is owned
    by slot (u mod n*C) div C (C = R*T*4 units) and summed in ring order from its owner (own,
    owner+1, ...; calVector(data, tmp) with tmp = own first)."""
    nw = (nbytes + 15) // 16 * 4
    padded = []
    for a in ins:
        w = np.zeros(nw, np.uint32)
        w.view(np.uint8)[:nbytes] = a.view(np.uint8)[:nbytes]
        padded.append(w)
    C = R * T * 4
    owner = ((np.arange(nw) // 4) % (n * C)) // C
    exp = np.zeros(nw, np.uint32)
    for o in range(n):
        order = [padded[(o + k) % n] for k in range(n)]
        seq = O.reduce_seq(dt, op, order)
        exp[owner == o] = seq[owner == o]
    return exp


@pytest.mark.parametrize("n,dt,count,R,T,stages", [
    (2, O.F16, 1 << 16, 2, 64, 2), (4, O.F16, (1 << 18) + 7, 2, 64, 2), (8, O.F16, 1 << 19, 2, 64, 3),
    (8, O.BF16, 100001, 4, 64, 2), (8, O.F32, 1 << 18, 2, 128, 2), (3, O.I32, 77777, 2, 64, 2),
    (8, O.F16, 1001, 2, 64, 1), (8, O.F16, 24 << 20, 32, 512, 64)])
def test_rsag_pipeline_bit_exact(built, n, dt, count, R, T, stages):
    """Pipelined RS+AG: outputs bit-exact against the ring-order oracle on the kernel's interleaved
    ownership; small workgroup counts and a scratch of only 1-3 stages force many iterations through
    the circular scratch (credits, put/reduce/recv hand-offs); the last case is the 48 MiB bucket."""
    import mscclpp_amd as m

    nbytes = count * ITEM[dt]
    C = R * T * 4
    stage = 2 * n * C * 16
    ranks = m.InProcessRanks(n, 1 << 16, bulk_scratch_bytes=stages * stage)
    for call in range(2):
        ins = _inputs(dt, n, count, seq=call, special=(call == 1 and dt in (O.F16, O.BF16)))
        dins = [_dev(a, dt) for a in ins]
        douts = [torch.full_like(d, 0) for d in dins]
        ranks.all_reduce(dins, douts, m.ALGO_RSAG_PIPELINE, op=O.SUM, nblocks=R, nthreads=T)
        torch.cuda.synchronize()
        assert ranks.errors() == [0] * n
        exp = _pipeline_expected(dt, O.SUM, ins, nbytes, n, R, T)
        for r in range(n):
            _cmp(_bytes(douts[r]), exp.view(np.uint8)[:nbytes], dt)


def test_rsag_pipeline_min(built):
    import mscclpp_amd as m

    n, dt, count, R, T = 4, O.F16, 50000, 2, 64
    ranks = m.InProcessRanks(n, 1 << 16, bulk_scratch_bytes=2 * 2 * n * R * T * 4 * 16)
    ins = _inputs(dt, n, count, seq=5)
    dins = [_dev(a, dt) for a in ins]
    douts = [torch.full_like(d, 0) for d in dins]
    ranks.all_reduce(dins, douts, m.ALGO_RSAG_PIPELINE, op=O.MIN, nblocks=R, nthreads=T)
    torch.cuda.synchronize()
    assert ranks.errors() == [0] * n
    exp = _pipeline_expected(dt, O.MIN, ins, count * 2, n, R, T)
    for r in range(n):
        _cmp(_bytes(douts[r]), exp.view(np.uint8)[: count * 2], dt)


def test_packet_grid_narrower_than_peers_is_invalid(built):
    """allreduce_packet.cu:238-241: an explicit LL16 grid with fewer workgroups than peers is an
    invalid argument (ncclInvalidArgument / CommInvalidArgument), not silently widened."""
    import mscclpp_amd as m

    n, count = 4, 4096
    ranks = m.InProcessRanks(n, m.scratch_required(m.ALGO_PACKET, n, count * 2, O.F16))
    ins = [torch.ones(count, dtype=torch.float16, device="cuda") for _ in range(n)]
    outs = [torch.empty_like(t) for t in ins]
    with pytest.raises(m.MscclppError) as e:
        ranks.all_reduce(ins, outs, m.ALGO_PACKET, nblocks=2, nthreads=256)
    assert e.value.code == 4
    ranks.all_reduce(ins, outs, m.ALGO_PACKET, nblocks=3, nthreads=256)  # = peers: accepted
    torch.cuda.synchronize()
    assert ranks.errors() == [0] * n and all(bool(torch.all(o == n)) for o in outs)
