"""Pin the C oracle (oracle/ll_oracle.c) against the numpy golden fixtures and the reference KATs.

Fixtures: tests/golden/golden_v1.npz, produced by tests/golden/make_golden.py (numpy only).
"""
import os

import numpy as np
import pytest

import oracle_lib as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden_v1.npz")


@pytest.fixture(scope="module")
def g():
    return np.load(GOLD, allow_pickle=False)


def _vec(fn, a, b):
    return np.array([fn(int(x), int(y)) for x, y in zip(a, b)], dtype=a.dtype)


def test_f16_add_and_min(g):
    assert np.array_equal(_vec(O.L().oracle_f16_add, g["f16_a"], g["f16_b"]), g["f16_add"])
    assert np.array_equal(_vec(O.L().oracle_f16_min, g["f16_a"], g["f16_b"]), g["f16_min"])


def test_bf16_add_and_min(g):
    assert np.array_equal(_vec(O.L().oracle_bf16_add, g["bf16_a"], g["bf16_b"]), g["bf16_add"])
    assert np.array_equal(_vec(O.L().oracle_bf16_min, g["bf16_a"], g["bf16_b"]), g["bf16_min"])


def test_f32_add_and_min(g):
    got = _vec(O.L().oracle_f32_add, g["f32_a"], g["f32_b"])
    exp = g["f32_add"]
    nan = (exp & 0x7FFFFFFF) > 0x7F800000
    assert np.array_equal(got[~nan], exp[~nan])
    assert np.all((got[nan] & 0x7FFFFFFF) > 0x7F800000)
    got = _vec(O.L().oracle_f32_min, g["f32_a"], g["f32_b"])
    exp = g["f32_min"]
    nan = (exp & 0x7FFFFFFF) > 0x7F800000
    # fminf tie on +-0 is implementation-defined; compare values there
    assert np.array_equal(got.view(np.float32)[~nan] == exp.view(np.float32)[~nan], np.ones((~nan).sum(), bool))


def test_clip_semantics_f16():
    L = O.L()
    assert L.oracle_f16_add(0x7BFF, 0x7BFF) == 0x7BFF  # 65504 + 65504 saturates
    assert L.oracle_f16_add(0x7C00, 0x3C00) == 0x7BFF  # +inf -> 65504
    assert L.oracle_f16_add(0xFC00, 0x3C00) == 0xFBFF  # -inf -> -65504
    assert L.oracle_f16_add(0x7E00, 0x3C00) == 0xFBFF  # NaN -> -65504 (hmax picks the bound)
    assert L.oracle_f16_add(0x0001, 0x0001) == 0x0002  # subnormals preserved
    assert L.oracle_bf16_add(0x7FC0, 0x3F80) == 0xFF80  # bf16 NaN -> -inf
    assert L.oracle_bf16_add(0x7F80, 0x3F80) == 0x7F80  # bf16 inf stays inf


def test_lcg_matches_reference_generator(g):
    assert np.array_equal(O.lcg(O.F16, 1000, 3, 1), g["lcg_f16_r3_s1"])
    assert np.array_equal(O.lcg(O.BF16, 1000, 3, 1), g["lcg_bf16_r3_s1"])
    assert np.array_equal(O.lcg(O.F32, 1000, 3, 1), g["lcg_f32_r3_s1"])


def test_packet_images(g):
    assert np.array_equal(O.ll16_pack(g["pkt_words"], 7), g["pkt_ll16_flag7"])
    assert np.array_equal(O.ll8_pack(g["pkt_words"], 7), g["pkt_ll8_flag7"])


def test_self_reduce(g):
    pk, out = O.self_reduce(O.F16, O.SUM, g["self_x"], g["self_y"], 1)
    assert np.array_equal(pk, g["self_pkts"])
    assert np.array_equal(out, g["self_out"])


def test_collectives_against_golden(g):
    k = 0
    while f"coll{k}_meta" in g:
        algo, n, dt, count, flag, half = [int(v) for v in g[f"coll{k}_meta"]]
        ins = list(g[f"coll{k}_in"])
        if algo == 0:
            outs, scr = O.allreduce_packet(dt, O.SUM, ins, count, flag, half)
        else:
            outs, scr = O.allreduce_allpairs(dt, O.SUM, ins, count, flag, half)
        exp_out = g[f"coll{k}_out"]
        W = exp_out.shape[1]
        for r in range(n):
            assert np.array_equal(outs[r][:W], exp_out[r]), (k, r)
            assert np.array_equal(scr[r], g[f"coll{k}_scratch"][r]), (k, r)
        k += 1
    assert k == 24


def test_bulk_orders_against_golden(g):
    for kind in (0, 1, 2):
        for dt in (O.F32, O.F16):
            ins = list(g[f"bulk{kind}_{dt}_in"])
            outs = O.allreduce_sliced(dt, O.SUM, ins, 8 * 96, 96, kind)
            for o in outs:
                assert np.array_equal(o, g[f"bulk{kind}_{dt}_out"])


def test_int32_kat():
    # allreduce_test.cu:1172-1183: input = rank, expected n(n-1)/2
    for n in (2, 4, 8):
        ins = [np.full(64, r, np.uint32) for r in range(n)]
        outs = O.allreduce_sliced(O.I32, O.SUM, ins, 64, 8, 0)
        assert all(np.all(o == n * (n - 1) // 2) for o in outs)
        outs, _ = O.allreduce_packet(O.I32, O.SUM, ins, 64, 1, 1 << 14)
        assert all(np.all(o[:64] == n * (n - 1) // 2) for o in outs)


def test_trigger_encoding(g):
    for row in g["triggers"]:
        typ, dst_id, dst_off, src_id, src_off, nbytes, sem, fst, snd = [int(v) for v in row]
        assert O.trigger_encode(typ, dst_id, dst_off, src_id, src_off, nbytes, sem) == (fst, snd)


def test_fifo_commit_parity():
    # fifo_device.hpp:120 / fifo_tests.cu:127-153: lap 0 writes 1, lap 1 writes 0, ...
    L = O.L()
    for pos in range(0, 4 * 512, 37):
        assert L.oracle_fifo_commit_bit(pos, 9) == ((pos >> 9) & 1) ^ 1


def test_bench_allreduce2_typed_restatement():
    """oracle_bench_allreduce2 (python/mscclpp_benchmark/allreduce.cu:223-289 for TYPE = int, float,
    __half): for int it is allreduce6's restatement word for word (same packets, same scratch image);
    for float / half its sum is 0 + peers ascending + own, unclipped -- an all-(-0) lane comes out +0
    where the own-first order keeps -0, half-ulp peers survive only when added before the owner's
    1.0 (n >= 3), and +-40000 halves overflow to inf instead of clipping to 65504."""
    n, nwords, flag = 4, 64, 3
    sb = 32 * nwords
    rng = np.random.default_rng(11)
    ins = [rng.integers(0, 2 ** 32, nwords, dtype=np.uint64).astype(np.uint32) for _ in range(n)]
    a, sa = O.bench_allreduce2(O.I32, ins, nwords, flag, sb)
    b, sbimg = O.mscclpp_test_ll(ins, nwords, flag, sb)
    for r in range(n):
        assert np.array_equal(a[r], b[r]) and np.array_equal(sa[r], sbimg[r])
    # float16: word w holds halves 2w, 2w+1; owner of word w = w // (nwords / n)
    epr = nwords // n
    h = [np.zeros(2 * nwords, np.float16) for _ in range(n)]
    for r in range(n):
        h[r][0::2] = -0.0  # low half of every word: -0 everywhere
        h[r][1::2] = np.float16(2.0 ** -11)  # high half: half an ulp of 1.0 ...
        for w in range(nwords):
            if w // epr == r:
                h[r][2 * w + 1] = np.float16(1.0)  # ... and 1.0 on the owner
    hw = [x.view(np.uint32) for x in h]
    o0, _ = O.bench_allreduce2(O.F16, hw, nwords, 1, sb, order=0)
    o1, _ = O.bench_allreduce2(O.F16, hw, nwords, 1, sb, order=1)
    for r in range(n):
        lo0, hi0 = o0[r].view(np.uint16)[0::2], o0[r].view(np.float16)[1::2]
        lo1, hi1 = o1[r].view(np.uint16)[0::2], o1[r].view(np.float16)[1::2]
        assert np.all(lo0 == 0x0000) and np.all(lo1 == 0x8000)  # +0 vs -0
        # 3 peers: 3 * 2^-11 exactly, then + 1.0 = 1 + 1.5 ulp, a tie that rounds to even: 1 + 2^-9
        assert np.all(hi0 == np.float16(1.0 + 2.0 ** -9))
        assert np.all(hi1 == np.float16(1.0))
    big = [np.full(2 * nwords, 40000.0, np.float16).view(np.uint32) for _ in range(2)]
    o, _ = O.bench_allreduce2(O.F16, big, nwords, 1, sb)
    assert np.all(o[0].view(np.uint16) == 0x7C00)  # inf, not clipped to 65504
    f = [np.full(nwords, -0.0, np.float32).view(np.uint32) for _ in range(2)]
    o, _ = O.bench_allreduce2(O.F32, f, nwords, 1, sb)
    assert np.all(o[0] == 0) and np.all(o[1] == 0)


def test_bench_allreduce1_restatement():
    """oracle_bench_allreduce1 (allreduce.cu:123-221): int32 gives the wrapping sum on every rank; for
    half the owner's value comes first -- an all-(-0) lane stays -0 (allreduce2's leading 0 makes it
    +0) -- and the peers follow in rotated channel order (rank r starts at channel r mod (n - 1))."""
    n, nwords = 4, 64
    rng = np.random.default_rng(5)
    ins = [rng.integers(0, 2 ** 32, nwords, dtype=np.uint64).astype(np.uint32) for _ in range(n)]
    out = O.bench_allreduce1(O.I32, ins, nwords)
    want = (np.sum(np.stack([a.astype(np.uint64) for a in ins]), axis=0) % (1 << 32)).astype(np.uint32)
    assert all(np.array_equal(o, want) for o in out)
    h = [np.full(2 * nwords, -0.0, np.float16).view(np.uint32) for _ in range(n)]
    assert all(np.all(o == 0x80008000) for o in O.bench_allreduce1(O.F16, h, nwords))
    # rotation: owner 1 of 3 ranks adds rank 2 before rank 0 (channel 1 then channel 0)
    n, cw = 3, 4
    vals = {0: 2.0 ** -11, 1: 1.0, 2: 2.0 ** -11}  # owner 1.0, the two peers half an ulp each
    f = [np.zeros(2 * n * cw, np.float16) for _ in range(n)]
    for q in range(n):
        f[q][:] = vals[q]
    out = O.bench_allreduce1(O.F16, [x.view(np.uint32) for x in f], n * cw)
    # owner-first: 1 + 2^-11 ties to 1 twice, whichever peer comes first
    assert np.all(out[0].view(np.float16)[2 * cw:4 * cw] == np.float16(1.0))
