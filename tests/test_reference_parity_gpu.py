"""GPU parity against the reference's OWN device code (oracle/_ref/libref.so, built from
/root/reference/include by oracle/build_ref.sh): LL16 packets via copyToPackets<LL16Packet>,
LL16Packet::read, and the f16x2 / bf16x2 / f32x2 operator+ / min with clip.

Both our product kernel and the reference harness run on the same random bit patterns
(NaN, inf, subnormals included); outputs and packet images must be bit-identical.  The CPU
oracle is checked against the reference harness too, which pins the oracle on the device."""
import ctypes
import os

import numpy as np
import pytest
import torch

import oracle_lib as O

pytestmark = pytest.mark.gpu

REF_SO = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref", "libref.so")


@pytest.fixture(scope="module")
def ref():
    if not os.path.exists(REF_SO):
        pytest.skip("oracle/_ref/libref.so not built (needs /root/reference at build time)")
    import mscclpp_amd  # noqa: F401  (torch + HIP runtime first)

    L = ctypes.CDLL(REF_SO)
    vp = ctypes.c_void_p
    L.refSelfReduceLL16.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, vp, vp, ctypes.c_uint64, ctypes.c_uint32, vp]
    L.refReduceWords.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, ctypes.c_size_t, vp]
    L.refPack.argtypes = [ctypes.c_int, vp, vp, ctypes.c_uint64, ctypes.c_uint32, vp]
    return L


def _words(n, seed):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)


def _dev_words(w):
    return torch.from_numpy(w.view(np.int32).copy()).cuda()


@pytest.mark.parametrize("dt,op", [(O.F16, O.SUM), (O.BF16, O.SUM), (O.F32, O.SUM), (O.I32, O.SUM),
                                   (O.F16, O.MIN), (O.BF16, O.MIN), (O.F32, O.MIN), (O.I32, O.MIN)])
def test_self_reduce_matches_reference_device_code(built, ref, dt, op):
    import mscclpp_amd as m

    nbytes = 1 << 20
    x, y = _words(nbytes // 4, 1), _words(nbytes // 4, 2)
    # signed zeros in both orders (min(-0, +0) = -0 on the device)
    x[:64], y[:64] = 0x80000000, 0
    x[64:128], y[64:128] = 0, 0x80000000
    x[128:192], y[128:192] = 0x80008000, 0x00000000
    xd, yd = _dev_words(x), _dev_words(y)
    # reference harness
    rpk = m.DeviceBuffer(2 * nbytes)
    rout = torch.zeros_like(xd)
    s = m.stream_ptr()
    assert ref.refSelfReduceLL16(dt, op, ctypes.c_void_p(xd.data_ptr()), ctypes.c_void_p(yd.data_ptr()),
                                 ctypes.c_void_p(rpk.ptr), ctypes.c_void_p(rout.data_ptr()), nbytes, 1, s) == 0
    # product kernel, same flag (1)
    tdt = {O.F16: torch.float16, O.BF16: torch.bfloat16, O.F32: torch.float32, O.I32: torch.int32}[dt]
    pk = m.DeviceBuffer(2 * nbytes)
    out = torch.zeros_like(xd)
    flags = torch.ones(m.FLAG_SLOTS, dtype=torch.int32, device="cuda")
    err = torch.zeros(16, dtype=torch.int32, device="cuda")
    m.self_reduce_ll16(xd.view(tdt), yd.view(tdt), pk.ptr, out.view(tdt), flags, err, op=op)
    torch.cuda.synchronize()
    assert int(err[0].item()) == 0
    got_w = out.cpu().numpy().view(np.uint32)
    ref_w = rout.cpu().numpy().view(np.uint32)
    if dt == O.F32 and op == O.SUM:
        # NaN + x: LLVM may commute an fadd, so which NaN operand's payload survives is the
        # compiler's choice per instantiation (the reference's own code is no exception): NaN words
        # must be NaN on both sides, every other word bit-identical
        nan = (ref_w & 0x7FFFFFFF) > 0x7F800000
        assert np.all((got_w[nan] & 0x7FFFFFFF) > 0x7F800000), "a NaN of the reference is not NaN here"
        bad = np.nonzero(got_w[~nan] != ref_w[~nan])[0]
    else:
        bad = np.nonzero(got_w != ref_w)[0]
    assert bad.size == 0, f"{bad.size} sum words differ from the reference's device code, first {bad[:4]}"
    got_pk = m.device_view(pk.ptr, 2 * nbytes)
    ref_pk = m.device_view(rpk.ptr, 2 * nbytes)
    assert torch.equal(got_pk, ref_pk), "LL16 packet image differs from copyToPackets<LL16Packet>"
    # and the CPU oracle agrees with the reference device code (f32 NaN payloads excepted)
    _, exp = O.self_reduce(dt, op, x, y, 1)
    r = rout.cpu().numpy().view(np.uint32)
    if dt == O.F32:
        nan = (r & 0x7FFFFFFF) > 0x7F800000
        assert np.array_equal(r[~nan], exp[~nan])
        assert np.all((exp[nan] & 0x7FFFFFFF) > 0x7F800000)
    else:
        assert np.array_equal(r, exp)
    rpk.free()
    pk.free()


def test_ll8_pack_matches_reference(built, ref):
    import mscclpp_amd as m

    nbytes = 64 << 10
    w = _words(nbytes // 4, 3)
    wd = _dev_words(w)
    rpk = m.DeviceBuffer(2 * nbytes)
    assert ref.refPack(1, ctypes.c_void_p(rpk.ptr), ctypes.c_void_p(wd.data_ptr()), nbytes, 9, m.stream_ptr()) == 0
    torch.cuda.synchronize()
    got = m.device_view(rpk.ptr, 2 * nbytes).cpu().numpy().view(np.uint32)
    assert np.array_equal(got, O.ll8_pack(w, 9))
    rpk.free()
