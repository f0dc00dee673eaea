"""GPU parity of the 1-byte reduce types the reference dispatches besides OCP FP8 (dispatchByDtype,
common.hpp:103-135): uint8 (Adapter<Op, uint8_t, uint8_t>) and the software float8 e4m3b15
accumulated in itself, half or float (dispatchFp8Accum).

1. The reference's own e4m3b15 conversions -- scalar and x4 paths -- and its calVectorAccum
   arithmetic for both types, compiled from /root/reference/include for gfx950
   (oracle/_ref/libref.so), pin the CPU oracle bit-exactly over every byte value; the conversions
   also meet the reference's unit-test known answers (tests/golden/e4m3b15_reference_kat.json).
2. The product kernels (self-reduce, LL16 two-hop, LL8 one-hop, bulk fullmesh / rsag / zero-copy)
   match the oracle bit-exactly on arbitrary bytes, packet images included.
3. ncclAllReduce with ncclUint8 (datatype_conversion.hpp:21-22) through the communicator of two
   processes, bit-exact."""
import ctypes
import json
import multiprocessing as mp
import os
import traceback

import numpy as np
import pytest
import torch

import mp_util
import oracle_lib as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref.so")
TYPES = (O.U8, O.B15, O.B15_ACC_F16, O.B15_ACC_F32)


@pytest.fixture(scope="module")
def ref():
    if not os.path.exists(REF_SO):
        pytest.skip("oracle/_ref/libref.so not built (needs /root/reference at build time)")
    import mscclpp_amd  # noqa: F401

    L = ctypes.CDLL(REF_SO)
    vp = ctypes.c_void_p
    L.refFp8Accum.argtypes = [ctypes.c_int, ctypes.c_int, vp, ctypes.c_int, ctypes.c_size_t, vp, vp]
    L.refB15Convert.argtypes = [vp, ctypes.c_size_t, vp, vp, vp, vp, vp]
    return L


def _vp(t):
    return ctypes.c_void_p(t.data_ptr())


def test_e4m3b15_conversions_match_reference(built, ref):
    """__fp8_e4m3b15(float), to<f8_e4m3b15x4>(f32x4), float(b15) and to<f32x4> as the reference runs
    them on gfx950, against the oracle and the reference unit test's known answers."""
    import mscclpp_amd as m

    kat = json.load(open(os.path.join(ROOT, "tests", "golden", "e4m3b15_reference_kat.json")))
    kin = [float.fromhex(x) if x not in ("inf", "-inf", "nan") else float(x) for x in kat["encode"]["inputs_hex"]]
    rng = np.random.default_rng(11)
    xs = np.concatenate([np.array(kin, np.float32), rng.uniform(-2.5, 2.5, 8000).astype(np.float32),
                         rng.uniform(-1e-3, 1e-3, 4000).astype(np.float32),
                         np.ldexp(1.0, np.arange(-26, 4)).astype(np.float32),
                         np.array([65504.0, 65520.0, -70000.0, 3e38], np.float32)])
    xs = np.concatenate([xs, np.zeros((-xs.size) % 4, np.float32)])
    n = xs.size
    din = torch.from_numpy(xs).cuda()
    enc = torch.zeros(n, dtype=torch.uint8, device="cuda")
    enc4 = torch.zeros_like(enc)
    dec = torch.zeros(256, dtype=torch.float32, device="cuda")
    dec4 = torch.zeros_like(dec)
    assert ref.refB15Convert(_vp(din), n, _vp(enc), _vp(enc4), _vp(dec), _vp(dec4), m.stream_ptr()) == 0
    torch.cuda.synchronize()
    exp = np.array([O.b15_encode(float(x)) for x in xs], np.uint8)
    for got in (enc.cpu().numpy(), enc4.cpu().numpy()):
        bad = np.nonzero(got != exp)[0]
        assert bad.size == 0, [(float(xs[i]), hex(got[i]), hex(exp[i])) for i in bad[:10]]
        assert list(got[: len(kin)]) == kat["encode"]["expected"]
    expd = np.array([O.b15_decode(b) for b in range(256)], np.float32).view(np.uint32)
    for got in (dec.cpu().numpy().view(np.uint32), dec4.cpu().numpy().view(np.uint32)):
        assert np.array_equal(got, expd)


@pytest.mark.parametrize("dt", TYPES)
@pytest.mark.parametrize("op", [O.SUM, O.MIN])
@pytest.mark.parametrize("nsrc", [2, 8])
def test_byte_type_accumulation_matches_reference(built, ref, dt, op, nsrc):
    """calVectorAccum over nsrc sources (every byte value) as the reference computes it vs the oracle."""
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


def _dev(arr):
    return torch.from_numpy(np.ascontiguousarray(arr, np.uint8).copy()).cuda()


def _bytes(t):
    return t.view(torch.uint8).cpu().numpy()


@pytest.mark.parametrize("dt", TYPES)
def test_byte_type_self_reduce(built, dt):
    import mscclpp_amd as m

    nbytes = 1 << 20
    rng = np.random.default_rng(dt)
    x = rng.integers(0, 256, nbytes, dtype=np.uint16).astype(np.uint8)
    y = rng.integers(0, 256, nbytes, dtype=np.uint16).astype(np.uint8)
    xd, yd = _dev(x), _dev(y)
    out = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
    pk = m.DeviceBuffer(2 * nbytes)
    flags = torch.ones(m.FLAG_SLOTS, dtype=torch.int32, device="cuda")
    err = torch.zeros(16, dtype=torch.int32, device="cuda")
    try:
        for op in (O.SUM, O.MIN):
            m.self_reduce_ll16(xd, yd, pk.ptr, out, flags, err, op=op, accum=dt)
            torch.cuda.synchronize()
            assert int(err[0].item()) == 0
            exp_pk, exp = O.self_reduce(dt, op, x, y, 1 + op)
            got, want = _bytes(out), exp.view(np.uint8)
            bad = np.nonzero(got != want)[0]
            assert bad.size == 0, (f"op {op}: {bad.size} mismatches: " + ", ".join(
                f"x=0x{x[i]:02x} y=0x{y[i]:02x} got=0x{got[i]:02x} oracle=0x{want[i]:02x}" for i in bad[:12]))
            assert np.array_equal(m.device_view(pk.ptr, 2 * nbytes).cpu().numpy().view(np.uint32), exp_pk)
    finally:
        pk.free()


def _inputs(dt, n, count, seq):
    rng = np.random.default_rng(2000 + 10 * dt + seq)
    return [rng.integers(0, 256, count, dtype=np.uint16).astype(np.uint8) for _ in range(n)]


LL_CASES = [(8, O.U8, 16384), (8, O.B15, 16384), (8, O.B15_ACC_F32, 8192), (4, O.B15_ACC_F16, 4096),
            (8, O.U8, 1001), (3, O.B15, 1002), (8, O.B15_ACC_F16, 7), (2, O.U8, 6)]


@pytest.mark.parametrize("algo", ["packet", "allpair"])
@pytest.mark.parametrize("n,dt,count", LL_CASES)
def test_byte_type_ll_allreduce_bit_exact(built, algo, n, dt, count):
    import mscclpp_amd as m

    code = m.ALGO_PACKET if algo == "packet" else m.ALGO_ALLPAIR
    sb = max(m.scratch_required(code, n, count, dt), 1 << 16)
    ranks = m.InProcessRanks(n, sb)
    for call, flag in enumerate((1, 2)):
        op = O.SUM if call == 0 else O.MIN
        ins = _inputs(dt, n, count, call)
        dins = [_dev(a) for a in ins]
        douts = [torch.zeros(count, dtype=torch.uint8, device="cuda") for _ in range(n)]
        ranks.all_reduce(dins, douts, code, op=op, nblocks=(n - 1) * 2 if algo == "packet" else 4, nthreads=256,
                         accum=dt)
        torch.cuda.synchronize()
        assert ranks.errors() == [0] * n
        fn = O.allreduce_packet if algo == "packet" else O.allreduce_allpairs
        exp, scr = fn(dt, op, ins, count, flag, sb // 2)
        for r in range(n):
            bad = np.nonzero(_bytes(douts[r]) != exp[r].view(np.uint8)[:count])[0]
            assert bad.size == 0, f"rank {r}: {bad.size} byte mismatches, first {bad[:8]}"
        if call == 0:
            for r in range(n):
                img = ranks.scratch_tensor(r, sb).cpu().numpy().view(np.uint32)
                assert np.array_equal(img, scr[r]), f"scratch image of rank {r}"


@pytest.mark.parametrize("algo,order", [("fullmesh", 0), ("rsag", 1), ("rsag_zc", 1)])
@pytest.mark.parametrize("n,dt,count", [(8, O.U8, 1 << 18), (8, O.B15_ACC_F32, 100000), (4, O.B15_ACC_F16, 65536 + 16),
                                        (7, O.B15, 12345), (8, O.U8, 4096)])
def test_byte_type_bulk_allreduce_bit_exact(built, algo, order, n, dt, count):
    import mscclpp_amd as m

    code = m.ALGO_NAMES[algo]
    slice_bytes = ((count + n - 1) // n + 15) // 16 * 16
    ranks = m.InProcessRanks(n, 1 << 16, bulk_scratch_bytes=max(n * slice_bytes, 1 << 20))
    for call in range(2):
        op = O.SUM if call == 0 else O.MIN
        ins = _inputs(dt, n, count, call)
        dins = [_dev(a) for a in ins]
        douts = [torch.zeros(count, dtype=torch.uint8, device="cuda") for _ in range(n)]
        ranks.all_reduce(dins, douts, code, op=op, nblocks=8, nthreads=256, accum=dt)
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
            bad = np.nonzero(_bytes(douts[r]) != exp[r].view(np.uint8)[:count])[0]
            assert bad.size == 0, f"rank {r}: {bad.size} byte mismatches, first {bad[:8]}"


def _u8_worker(rank, n, uid, q):
    try:
        os.environ.setdefault("MSCCLPP_AMD_SPIN_TIMEOUT_MS", "10000")
        import torch

        import mp_util
        import mscclpp_amd as m
        import oracle_lib as O

        mp_util.place_rank(rank, n)
        comm = m.Communicator(rank, n, uid)
        res = []
        for count in (4096, 1 << 20, (3 << 20) + 5):  # the LL8, LL16 and bulk ranges of the selector
            ins = [np.random.default_rng(50 + r).integers(0, 256, count, dtype=np.uint16).astype(np.uint8)
                   for r in range(n)]
            x = torch.from_numpy(ins[rank].copy()).cuda()
            y = torch.zeros_like(x)
            for op in ("sum", "min"):
                comm.all_reduce(x, y, op=op)  # ncclAllReduce(..., ncclUint8, ...)
                torch.cuda.synchronize()
                o = O.SUM if op == "sum" else O.MIN
                exp = O.reduce_seq(O.U8, o, [np.pad(a, (0, (-count) % 4)).view(np.uint32) for a in ins]).view(
                    np.uint8)[:count]  # wrapping add / min commute: one result in every order
                res.append((count, op, int(np.count_nonzero(y.cpu().numpy() != exp))))
        # ncclReduceScatter over uint8 (blocks of 16-byte multiples): rank r gets block r of the sum
        blk = 1 << 18
        ins = [np.random.default_rng(70 + r).integers(0, 256, n * blk, dtype=np.uint16).astype(np.uint8)
               for r in range(n)]
        x = torch.from_numpy(ins[rank].copy()).cuda()
        y = torch.zeros(blk, dtype=torch.uint8, device="cuda")
        comm.reduce_scatter(x, y, op="sum")
        torch.cuda.synchronize()
        exp = O.reduce_seq(O.U8, O.SUM, [a.view(np.uint32) for a in ins]).view(np.uint8)[rank * blk:(rank + 1) * blk]
        res.append(("rs", "sum", int(np.count_nonzero(y.cpu().numpy() != exp))))
        err = comm.device_error()
        comm.destroy()
        q.put((rank, {"res": res, "err": err}, None))
    except Exception:
        q.put((rank, None, traceback.format_exc()))


def test_nccl_uint8_two_processes(built):
    """ncclAllReduce (LL8, LL16 and bulk sizes, SUM and MIN) and ncclReduceScatter over ncclUint8."""
    import mscclpp_amd as m

    n = 2
    uid = m.Communicator.unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_u8_worker, args=(r, n, uid, q)) for r in range(n)]
    for p in procs:
        p.start()
    got = mp_util.collect(procs, q, n, 240)
    for rank, r in got.items():
        assert r["err"] == 0 and all(bad == 0 for _, _, bad in r["res"]), (rank, r)
