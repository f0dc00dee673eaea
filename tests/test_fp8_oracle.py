"""CPU checks of the oracle's OCP FP8 arithmetic against torch's independent
float8_e4m3fn / float8_e5m2 conversions and numpy float16 / float32 accumulation.

The reference's gfx950 arithmetic (gpu_data_types.hpp:353-750 generic branches, reduce_kernel.hpp:
139-189, amd_hip_fp8.h:548-592) is: decode exactly, accumulate in AccumT, encode with saturation to
the largest finite value and round-to-nearest-even.  torch rounds the same way inside the finite
range, so every finite case is pinned here; NaN / Inf images are pinned on the GPU against the
reference's own conversions (tests/test_fp8_gpu.py)."""
import numpy as np
import pytest
import torch

import oracle_lib as O

TF8 = {False: torch.float8_e4m3fn, True: torch.float8_e5m2}
MAXF = {False: 448.0, True: 57344.0}


def _torch_decode(b, e5):
    return torch.from_numpy(np.asarray(b, np.uint8)).view(TF8[e5]).float().numpy()


def _torch_encode(f, e5):
    f = np.clip(np.asarray(f, np.float32), -MAXF[e5], MAXF[e5])
    return torch.from_numpy(f).to(TF8[e5]).view(torch.uint8).numpy()


@pytest.mark.parametrize("e5", [False, True])
def test_decode_all_bytes(e5):
    ref = _torch_decode(np.arange(256), e5)
    got = np.array([O.fp8_decode(b, e5) for b in range(256)], np.float32)
    nan = np.isnan(ref)
    assert np.array_equal(np.isnan(got), nan)
    assert np.array_equal(got[~nan].view(np.uint32), ref[~nan].view(np.uint32))  # exact, signed zeros too


@pytest.mark.parametrize("e5", [False, True])
def test_encode_rne_and_saturation(e5):
    rng = np.random.default_rng(5)
    m = MAXF[e5]
    # every representable value, every midpoint between neighbours (ties -> even), random values
    # over the whole range including subnormals, and out-of-range values (saturate)
    vals = _torch_decode(np.arange(256), e5)
    vals = np.sort(vals[np.isfinite(vals)])
    mids = (vals[:-1].astype(np.float64) + vals[1:]) / 2
    rand = rng.standard_normal(20000).astype(np.float32) * np.float32(m / 8)
    tiny = rng.standard_normal(5000).astype(np.float32) * np.float32(2.0 ** (-14 if e5 else -6))
    big = np.array([m * 1.01, -m * 1.5, 1e30, -1e30, m + 1, -(m + 1)], np.float32)
    xs = np.concatenate([vals, mids.astype(np.float32), rand, tiny, big])
    got = np.array([O.fp8_encode_sat(x, e5) for x in xs], np.uint8)
    exp = _torch_encode(xs, e5)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, [(float(xs[i]), int(got[i]), int(exp[i])) for i in bad[:8]]


def _rand_fp8(rng, n, e5, finite=True):
    b = rng.integers(0, 256, n, dtype=np.uint16).astype(np.uint8)
    if finite:
        f = _torch_decode(b, e5)
        b[~np.isfinite(f)] = 0x38  # 1.0 in e4m3 / 0.5 in e5m2
    return b


@pytest.mark.parametrize("dt", O.FP8_TYPES)
@pytest.mark.parametrize("op", [O.SUM, O.MIN])
def test_reduce_seq_matches_numpy(dt, op):
    """calVectorAccum<T, AccumT> over 8 sources in order, finite inputs."""
    e5 = O.is_e5m2(dt)
    rng = np.random.default_rng(dt * 10 + op)
    n = 4096
    srcs = [_rand_fp8(rng, n, e5) for _ in range(8)]
    got = O.reduce_seq(dt, op, srcs).view(np.uint8)
    dec = [_torch_decode(s, e5) for s in srcs]
    if dt in (O.E4M3_ACC_F32, O.E5M2_ACC_F32):
        acc = dec[0].astype(np.float32)
        for d in dec[1:]:
            acc = acc + d if op == O.SUM else np.where(acc < d, acc, d)
        exp = _torch_encode(acc, e5)
    elif dt in (O.E4M3_ACC_F16, O.E5M2_ACC_F16):
        acc = dec[0].astype(np.float16)
        with np.errstate(over="ignore", invalid="ignore"):
            for d in dec[1:]:
                d16 = d.astype(np.float16)
                acc = (acc + d16) if op == O.SUM else np.where(acc < d16, acc, d16)
        a32 = acc.astype(np.float32)
        fin = np.isfinite(a32)
        exp = _torch_encode(np.where(fin, a32, 0), e5)
        # a half accumulator that overflowed to +-inf is converted without saturation (inf is
        # exempt from the clamp in amd_hip_fp8.h:561-575): e5m2 keeps inf, e4m3 has only NaN
        exp = np.where(fin, exp, np.where(a32 > 0, 0x7C if e5 else 0x7F, 0xFC if e5 else 0xFF)).astype(np.uint8)
    else:
        acc = srcs[0].copy()
        for s in srcs[1:]:
            a, b = _torch_decode(acc, e5), _torch_decode(s, e5)
            if op == O.MIN:
                acc = _torch_encode(np.fmin(a, b), e5)
            else:
                acc = _torch_encode(a + b, e5)  # saturating; e5m2 clip is then the identity on finite sums
        exp = acc
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, [(i, int(got[i]), int(exp[i])) for i in bad[:8]]


def test_e5m2_clip_turns_nan_into_min_finite():
    """clip<__fp8_e5m2> (gpu_data_types.hpp:362-371): fmaxf(NaN, -57344) = -57344."""
    nan, inf, one = 0x7F, 0x7C, 0x3C
    a = np.array([nan, inf, inf, one, nan, 0x7B], np.uint8)
    b = np.array([one, one, 0xFC, 0xFC, nan, 0x7B], np.uint8)
    got = O.reduce_seq(O.E5M2, O.SUM, [np.tile(a, 4)[:24].copy(), np.tile(b, 4)[:24].copy()]).view(np.uint8)[:6]
    # NaN -> -57344 (0xFB); inf + 1 = inf -> 57344 (0x7B); inf + -inf = NaN -> -57344; 1 + -inf -> -57344;
    # 57344 + 57344 saturates to 57344
    assert list(got) == [0xFB, 0x7B, 0xFB, 0xFB, 0xFB, 0x7B]


@pytest.mark.parametrize("dt,count", [(O.E4M3, 5), (O.E4M3, 6), (O.E4M3, 7), (O.E4M3, 8), (O.E5M2, 1), (O.F16, 3)])
def test_ll_words_cover_the_buffer(dt, count):
    w = O.ll_words(dt, count)
    assert w * 4 >= count * O.itemsize(dt)
    if O.itemsize(dt) == 1 and count % 4 in (0, 3):  # sizes the reference handles keep its count
        assert w == (count + 1) // 4
