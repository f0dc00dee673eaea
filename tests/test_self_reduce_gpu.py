"""GPU parity: the 1-GPU LL16 pack -> sum -> unpack kernel against the CPU oracle, bit-exact,
including the packet image (flag words and data words) left in the packet buffer."""
import numpy as np
import pytest
import torch

import oracle_lib as O

pytestmark = pytest.mark.gpu

TORCH = {O.F16: torch.float16, O.BF16: torch.bfloat16, O.F32: torch.float32, O.I32: torch.int32}


def _inputs(dt, nbytes, special):
    itemsize = 2 if dt in (O.F16, O.BF16) else 4
    count = nbytes // itemsize
    x = O.lcg(dt, count, 0, 0)
    y = O.lcg(dt, count, 1, 0)
    if special:
        rng = np.random.default_rng(7)
        bits = 16 if itemsize == 2 else 32
        m = rng.random(count) < 0.5
        x = x.copy()
        y = y.copy()
        x[m] = rng.integers(0, 2**bits, m.sum(), dtype=np.uint64).astype(x.dtype)
        y[m] = rng.integers(0, 2**bits, m.sum(), dtype=np.uint64).astype(y.dtype)
    return x, y


def _to_dev(arr, dt):
    t = torch.from_numpy(arr.view(np.int16 if arr.dtype == np.uint16 else np.int32).copy())
    return t.view(TORCH[dt]).cuda()


def _bits(t):
    return t.cpu().view(torch.int16 if t.element_size() == 2 else torch.int32).numpy().view(
        np.uint16 if t.element_size() == 2 else np.uint32)


def _assert_equal_words(got, exp, dt):
    got = got.view(np.uint32)
    exp = exp.view(np.uint32)
    if dt == O.F32:
        nan = (exp & 0x7FFFFFFF) > 0x7F800000
        assert np.array_equal(got[~nan], exp[~nan])
        assert np.all((got[nan] & 0x7FFFFFFF) > 0x7F800000)
    else:
        bad = np.nonzero(got != exp)[0]
        assert bad.size == 0, f"{bad.size} mismatches, first at {bad[:4]}: {got[bad[:4]]} vs {exp[bad[:4]]}"


@pytest.mark.parametrize("dt,op", [(O.F16, O.SUM), (O.BF16, O.SUM), (O.F32, O.SUM), (O.I32, O.SUM),
                                   (O.F16, O.MIN), (O.BF16, O.MIN), (O.F32, O.MIN)])
@pytest.mark.parametrize("nbytes,special", [
    (16, True), (1040, False), ((7 << 10) + 48, True),   # 1 KiB per wave, one round, ragged tails
    (64 << 10, True), ((1 << 20) + 48, False),
    (4 << 20, True),                                     # the largest one-round grid: 1024 workgroups
    ((4 << 20) + 16, False),                             # two rounds
    ((8 << 20) + 16, False),                             # three rounds and more: partner tiles one round late
    ((24 << 20) + 16, True),
    ((32 << 20) + 16, False)])                           # eight rounds and more: two rounds late
def test_self_reduce_bit_exact(built, dt, op, nbytes, special):
    import mscclpp_amd as m

    x, y = _inputs(dt, nbytes, special)
    xd, yd = _to_dev(x, dt), _to_dev(y, dt)
    out = torch.empty_like(xd)
    pk = m.DeviceBuffer(2 * nbytes)
    flags = torch.ones(m.FLAG_SLOTS, dtype=torch.int32, device="cuda")
    err = torch.zeros(16, dtype=torch.int32, device="cuda")
    for flag in (1, 2, 3):
        out.zero_()
        m.self_reduce_ll16(xd, yd, pk.ptr, out, flags, err, op=op)
        torch.cuda.synchronize()
        assert int(err[0].item()) == 0
        exp_pk, exp_out = O.self_reduce(dt, op, x, y, flag)
        _assert_equal_words(_bits(out), exp_out, dt)
        got_pk = m.device_view(pk.ptr, 2 * nbytes).cpu().numpy().view(np.uint32)
        assert np.array_equal(got_pk, exp_pk)  # LL16 flag and data words, bit-exact
        assert int(flags[0].item()) == flag + 1 and int(flags[-1].item()) == flag + 1
    pk.free()


def test_self_reduce_rejects_unaligned(built):
    import mscclpp_amd as m

    x = torch.zeros(9, dtype=torch.float16, device="cuda")
    flags = torch.ones(m.FLAG_SLOTS, dtype=torch.int32, device="cuda")
    err = torch.zeros(16, dtype=torch.int32, device="cuda")
    with pytest.raises(m.MscclppError) as e:
        m.self_reduce_ll16(x, x, x.data_ptr(), x, flags, err)
    assert e.value.code == 4


@pytest.mark.parametrize("nbytes,waves,nblocks,skew", [
    (16, 4, 2, 0), (1 << 20, 4, 256, 0), ((1 << 20) + 48, 8, 130, 0), (4 << 20, 8, 512, 0),
    ((4 << 20) + 16, 4, 1024, 1), ((8 << 20) + 16, 4, 1024, 1), ((24 << 20) + 16, 4, 1024, 1),
    ((32 << 20) + 16, 4, 1024, 2), (48 << 20, 4, 1024, 2)])
def test_self_reduce_default_shape(built, nbytes, waves, nblocks, skew):
    """The launch shape the product entry picks (4 waves x 1 KiB, one workgroup per 4 KiB up to 1024,
    8-wave workgroups for one round of 8 KiB tiles above 1 MiB up to 4 MiB, partner tiles consumed
    one round late from three rounds per workgroup on, two rounds late from eight)."""
    import ctypes

    import mscclpp_amd as m

    w, u, nb, sk = (ctypes.c_int() for _ in range(4))
    m.check(m.lib().mscclppAmdSelfReduceLL16DefaultShape(nbytes, ctypes.byref(w), ctypes.byref(u), ctypes.byref(nb),
                                                         ctypes.byref(sk)), "default shape")
    assert (w.value, u.value, nb.value, sk.value) == (waves, 1, nblocks, skew)



@pytest.mark.parametrize("nbytes", [8 << 10, (8 << 20) + (8 << 10)])
def test_self_reduce_stream_mirror_in_bounds(built, nbytes):
    """The benchmark's same-traffic ceiling kernel (mscclppAmdSelfReduceStream) stores every packet of
    the packet buffer (flag word 0) and nothing past the packet buffer or the output; sizes that are
    not a multiple of 8 KiB are rejected."""
    import mscclpp_amd as m

    guard = 1 << 16
    x = torch.randint(-2**15, 2**15, (nbytes // 2,), dtype=torch.int16, device="cuda")
    y = torch.randint(-2**15, 2**15, (nbytes // 2,), dtype=torch.int16, device="cuda")
    out = torch.full(((nbytes + guard) // 4,), -1, dtype=torch.int32, device="cuda")
    pk = torch.full(((2 * nbytes + guard) // 4,), -1, dtype=torch.int32, device="cuda")
    L = m.lib()
    m.check(L.mscclppAmdSelfReduceStream(x.data_ptr(), y.data_ptr(), pk.data_ptr(), out.data_ptr(), nbytes,
                                         m.stream_ptr()), "stream mirror")
    torch.cuda.synchronize()
    words = pk.cpu().numpy().view(np.uint32)
    flags = words[: 2 * nbytes // 4].reshape(-1, 4)[:, [1, 3]]
    assert np.all(flags == 0)  # every packet of the 2 * nbytes buffer was stored
    assert np.all(words[2 * nbytes // 4:] == 0xFFFFFFFF)
    assert np.all(out.cpu().numpy().view(np.uint32)[nbytes // 4:] == 0xFFFFFFFF)
    assert L.mscclppAmdSelfReduceStream(x.data_ptr(), y.data_ptr(), pk.data_ptr(), out.data_ptr(), nbytes - 4096,
                                        m.stream_ptr()) == 4
