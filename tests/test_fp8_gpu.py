"""GPU parity of the OCP FP8 reduce types (e4m3 / e5m2 with AccumT = T, half,
float; reduce_kernel.hpp:139-189, common.hpp:89-100).

1. The reference's own fp8 conversions and calVectorAccum arithmetic, compiled from
   /root/reference/include for gfx950 (oracle/_ref/libref.so), pin the CPU oracle bit-exactly,
   NaN / Inf / subnormal / saturation cases included.
2. The product kernels (self-reduce, LL16 two-hop, LL8 one-hop, bulk fullmesh / rsag) match the
   oracle bit-exactly, packet images included, on the same inputs."""
import ctypes
import os

import numpy as np
import pytest
import torch

import oracle_lib as O

pytestmark = pytest.mark.gpu

REF_SO = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref", "libref.so")
ELEM = {O.E4M3: torch.float8_e4m3fn, O.E5M2: torch.float8_e5m2, O.E4M3_ACC_F16: torch.float8_e4m3fn,
        O.E5M2_ACC_F16: torch.float8_e5m2, O.E4M3_ACC_F32: torch.float8_e4m3fn, O.E5M2_ACC_F32: torch.float8_e5m2}
ACC = {O.E4M3: None, O.E5M2: None, O.E4M3_ACC_F16: torch.float16, O.E5M2_ACC_F16: torch.float16,
       O.E4M3_ACC_F32: torch.float32, O.E5M2_ACC_F32: torch.float32}


@pytest.fixture(scope="module")
def ref():
    if not os.path.exists(REF_SO):
        pytest.skip("oracle/_ref/libref.so not built (needs /root/reference at build time)")
    import mscclpp_amd  # noqa: F401

    L = ctypes.CDLL(REF_SO)
    vp = ctypes.c_void_p
    L.refFp8Accum.argtypes = [ctypes.c_int, ctypes.c_int, vp, ctypes.c_int, ctypes.c_size_t, vp, vp]
    L.refFp8Convert.argtypes = [vp, ctypes.c_size_t, vp, vp, vp, vp, vp]
    return L


def _vp(t):
    return ctypes.c_void_p(t.data_ptr())


def _special_floats():
    m = []
    for v in (448.0, 464.0, 480.0, 57344.0, 61440.0, 65504.0, 1e9, 2.0 ** -6, 2.0 ** -9, 2.0 ** -10, 2.0 ** -14,
              2.0 ** -16, 2.0 ** -17, 1.5 * 2.0 ** -17, 0.0, 1.0, 1.0625, 1.125, 3.0 * 2 ** -10, 1e-30):
        m += [v, -v]
    f = np.array(m, np.float32)
    bits = np.array([0x7F800000, 0xFF800000, 0x7FC00000, 0xFFC00000, 0x7F800001, 0xFFBFFFFF], np.uint32)
    return np.concatenate([f, bits.view(np.float32)])


def test_fp8_conversions_match_reference(built, ref):
    """__fp8_e4m3(float) / __fp8_e5m2(float) and float(fp8) as the reference runs them on gfx950."""
    import mscclpp_amd as m

    rng = np.random.default_rng(7)
    xs = np.concatenate([_special_floats(), rng.standard_normal(4000).astype(np.float32) * 300,
                         rng.standard_normal(4000).astype(np.float32) * 0.01,
                         (rng.standard_normal(4000) * 3e4).astype(np.float32)])
    n = xs.size
    din = torch.from_numpy(xs).cuda()
    e4 = torch.zeros(n, dtype=torch.uint8, device="cuda")
    e5 = torch.zeros_like(e4)
    d4 = torch.zeros(256, dtype=torch.float32, device="cuda")
    d5 = torch.zeros_like(d4)
    assert ref.refFp8Convert(_vp(din), n, _vp(e4), _vp(e5), _vp(d4), _vp(d5), m.stream_ptr()) == 0
    torch.cuda.synchronize()
    report = []
    for e5m2, got_enc, got_dec in ((False, e4, d4), (True, e5, d5)):
        enc = got_enc.cpu().numpy()
        exp = np.array([O.fp8_encode_sat(x, e5m2) for x in xs], np.uint8)
        bad = np.nonzero(enc != exp)[0]
        report += [f"enc e5m2={e5m2} x={xs[i]!r} (0x{xs[i:i+1].view(np.uint32)[0]:08x}) ref=0x{enc[i]:02x} "
                   f"oracle=0x{exp[i]:02x}" for i in bad[:12]]
        dec = got_dec.cpu().numpy().view(np.uint32)
        expd = np.array([O.fp8_decode(b, e5m2) for b in range(256)], np.float32).view(np.uint32)
        badd = np.nonzero(dec != expd)[0]
        report += [f"dec e5m2={e5m2} byte=0x{b:02x} ref=0x{dec[b]:08x} oracle=0x{expd[b]:08x}" for b in badd[:12]]
    assert not report, "\n" + "\n".join(report)


@pytest.mark.parametrize("dt", O.FP8_TYPES)
@pytest.mark.parametrize("op", [O.SUM, O.MIN])
@pytest.mark.parametrize("nsrc", [2, 8])
def test_fp8_accumulation_matches_reference(built, ref, dt, op, nsrc):
    """calVectorAccum over nsrc sources (all 256 byte values, NaN / Inf included) vs the oracle."""
    import mscclpp_amd as m

    rng = np.random.default_rng(100 * dt + 10 * op + nsrc)
    nwords = 1 << 14
    src = rng.integers(0, 2 ** 32, (nsrc, nwords), dtype=np.uint64).astype(np.uint32)
    dsrc = torch.from_numpy(src.view(np.int32).copy()).cuda()
    dout = torch.zeros(nwords, dtype=torch.int32, device="cuda")
    assert ref.refFp8Accum(dt, op, _vp(dsrc), nsrc, nwords, _vp(dout), m.stream_ptr()) == 0
    torch.cuda.synchronize()
    got = dout.cpu().numpy().view(np.uint32).view(np.uint8)
    exp = O.reduce_seq(dt, op, [src[k] for k in range(nsrc)]).view(np.uint8)
    bad = np.nonzero(got != exp)[0]
    if bad.size:
        b = src.view(np.uint8).reshape(nsrc, -1)
        rows = [f"i={i} srcs={[hex(int(b[k, i])) for k in range(nsrc)]} ref=0x{got[i]:02x} oracle=0x{exp[i]:02x}"
                for i in bad[:10]]
        pytest.fail(f"{bad.size} mismatches\n" + "\n".join(rows))


def _fp8_dev(arr, dt):
    return torch.from_numpy(np.ascontiguousarray(arr, np.uint8).copy()).cuda().view(ELEM[dt])


def _bytes(t):
    return t.view(torch.uint8).cpu().numpy()


@pytest.mark.parametrize("dt", O.FP8_TYPES)
def test_fp8_self_reduce(built, dt):
    import mscclpp_amd as m

    nbytes = 1 << 20
    rng = np.random.default_rng(dt)
    x = rng.integers(0, 256, nbytes, dtype=np.uint16).astype(np.uint8)
    y = rng.integers(0, 256, nbytes, dtype=np.uint16).astype(np.uint8)
    xd, yd = _fp8_dev(x, dt), _fp8_dev(y, dt)
    out = torch.zeros(nbytes, dtype=torch.uint8, device="cuda").view(ELEM[dt])
    pk = m.DeviceBuffer(2 * nbytes)
    flags = torch.ones(m.FLAG_SLOTS, dtype=torch.int32, device="cuda")
    err = torch.zeros(16, dtype=torch.int32, device="cuda")
    for op in (O.SUM, O.MIN):
        m.self_reduce_ll16(xd, yd, pk.ptr, out, flags, err, op=op, accum=ACC[dt])
        torch.cuda.synchronize()
        assert int(err[0].item()) == 0
        flag = 1 + op
        exp_pk, exp = O.self_reduce(dt, op, x, y, flag)
        assert np.array_equal(_bytes(out), exp.view(np.uint8))
        assert np.array_equal(m.device_view(pk.ptr, 2 * nbytes).cpu().numpy().view(np.uint32), exp_pk)
    pk.free()


def _inputs(dt, n, count, seq):
    rng = np.random.default_rng(1000 + seq)
    ins = []
    for r in range(n):
        a = O.lcg(dt, count, r, seq).copy()
        msk = rng.random(count) < 0.2  # arbitrary bytes: NaN, Inf, subnormals, large values
        a[msk] = rng.integers(0, 256, msk.sum(), dtype=np.uint16).astype(np.uint8)
        ins.append(a)
    return ins


LL_CASES = [(8, O.E4M3, 16384), (8, O.E5M2, 16384), (8, O.E4M3_ACC_F32, 8192), (8, O.E5M2_ACC_F16, 8192),
            (4, O.E4M3_ACC_F16, 4096), (4, O.E5M2_ACC_F32, 4096), (8, O.E4M3, 1001), (3, O.E5M2_ACC_F32, 1002),
            (8, O.E4M3_ACC_F32, 7), (2, O.E5M2, 6)]


@pytest.mark.parametrize("algo", ["packet", "allpair"])
@pytest.mark.parametrize("n,dt,count", LL_CASES)
def test_fp8_ll_allreduce_bit_exact(built, algo, n, dt, count):
    import mscclpp_amd as m

    code = m.ALGO_PACKET if algo == "packet" else m.ALGO_ALLPAIR
    sb = max(m.scratch_required(code, n, count, dt), 1 << 16)
    ranks = m.InProcessRanks(n, sb)
    for call, flag in enumerate((1, 2)):
        op = O.SUM if call == 0 else O.MIN
        ins = _inputs(dt, n, count, call)
        dins = [_fp8_dev(a, dt) for a in ins]
        douts = [torch.zeros(count, dtype=torch.uint8, device="cuda").view(ELEM[dt]) for _ in range(n)]
        ranks.all_reduce(dins, douts, code, op=op, nblocks=(n - 1) * 2 if algo == "packet" else 4, nthreads=256,
                         accum=ACC[dt])
        torch.cuda.synchronize()
        assert ranks.errors() == [0] * n
        if algo == "packet":
            exp, scr = O.allreduce_packet(dt, op, ins, count, flag, sb // 2)
        else:
            exp, scr = O.allreduce_allpairs(dt, op, ins, count, flag, sb // 2)
        for r in range(n):
            got = _bytes(douts[r])
            bad = np.nonzero(got != exp[r].view(np.uint8)[:count])[0]
            assert bad.size == 0, f"rank {r}: {bad.size} byte mismatches, first {bad[:8]}"
        if call == 0:
            for r in range(n):
                img = ranks.scratch_tensor(r, sb).cpu().numpy().view(np.uint32)
                assert np.array_equal(img, scr[r]), f"scratch image of rank {r}"


@pytest.mark.parametrize("algo,order", [("fullmesh", 0), ("rsag", 1), ("rsag_zc", 1)])
@pytest.mark.parametrize("n,dt,count", [(8, O.E4M3, 1 << 18), (8, O.E5M2_ACC_F32, 100000), (4, O.E4M3_ACC_F16, 65536 + 16),
                                        (7, O.E5M2, 12345), (8, O.E4M3_ACC_F32, 4096)])
def test_fp8_bulk_allreduce_bit_exact(built, algo, order, n, dt, count):
    import mscclpp_amd as m

    code = m.ALGO_NAMES[algo]
    slice_bytes = ((count + n - 1) // n + 15) // 16 * 16
    ranks = m.InProcessRanks(n, 1 << 16, bulk_scratch_bytes=max(n * slice_bytes, 1 << 20))
    for call in range(2):
        op = O.SUM if call == 0 else O.MIN
        ins = _inputs(dt, n, count, call)
        dins = [_fp8_dev(a, dt) for a in ins]
        douts = [torch.zeros(count, dtype=torch.uint8, device="cuda").view(ELEM[dt]) for _ in range(n)]
        ranks.all_reduce(dins, douts, code, op=op, nblocks=8, nthreads=256, accum=ACC[dt])
        torch.cuda.synchronize()
        assert ranks.errors() == [0] * n
        nwords = (count + 3) // 4
        padded = []
        for a in ins:
            w = np.zeros(nwords, np.uint32)
            w.view(np.uint8)[:count] = a
            padded.append(w)
        exp = O.allreduce_sliced(dt, op, padded, nwords, slice_bytes // 4, order)
        for r in range(n):
            got = _bytes(douts[r])
            bad = np.nonzero(got != exp[r].view(np.uint8)[:count])[0]
            assert bad.size == 0, f"rank {r}: {bad.size} byte mismatches, first {bad[:8]}"
