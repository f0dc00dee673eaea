"""The 1-byte reduce types the reference dispatches besides OCP FP8 (common.hpp:103-135): uint8 and
the software float8 e4m3b15 accumulated in itself, half or float.  CPU only.

* e4m3b15 conversions: the C oracle (oracle/ll_oracle.c b15_encode / b15_decode) against the
  reference's own known answers (tests/golden/e4m3b15_reference_kat.json, from
  test/unit/gpu_data_types_tests.cu:95-139), and against an independent numpy statement of
  gpu_data_types.hpp:111-155 for every byte and a sweep of floats.
* e4m3b15 and uint8 reductions: oracle_reduce_seq against numpy statements of the three
  accumulation forms (reduce_kernel.hpp:139-189; gpu_data_types.hpp:577-640, 1269-1300)."""
import json
import os

import numpy as np
import pytest

import oracle_lib as O

HERE = os.path.dirname(os.path.abspath(__file__))


def _np_b15_to_h16(b):
    b = np.asarray(b, np.uint16)
    return (((b & 0x80) << 8) | ((b & 0x7F) << 7)).astype(np.uint16)


def _np_b15_decode(b):
    return _np_b15_to_h16(b).view(np.float16).astype(np.float32)


def _np_b15_from_h16(h):
    h = np.asarray(h, np.uint16).astype(np.uint32)
    a = np.minimum(h & 0x7FFF, 0x3F80)
    return ((((a * 2 + 0x80) | (h & 0x8000)) >> 8) & 0xFF).astype(np.uint8)


def _np_b15_encode(f):
    with np.errstate(over="ignore", invalid="ignore"):
        h = np.asarray(f, np.float32).astype(np.float16).view(np.uint16)  # RNE, as __float2half_rn
    return _np_b15_from_h16(h)


def test_e4m3b15_reference_known_answers(built):
    kat = json.load(open(os.path.join(HERE, "golden", "e4m3b15_reference_kat.json")))
    vals = [float.fromhex(x) if x not in ("inf", "-inf", "nan") else float(x) for x in kat["encode"]["inputs_hex"]]
    assert [O.b15_encode(v) for v in vals] == kat["encode"]["expected"]
    want = [float.fromhex(x) for x in kat["decode"]["expected_hex"]]
    got = [O.b15_decode(b) for b in kat["decode"]["raw"]]
    assert [np.float32(g).tobytes() for g in got] == [np.float32(w).tobytes() for w in want]  # -0.0 too


def test_e4m3b15_every_byte_and_a_float_sweep_match_numpy(built):
    b = np.arange(256, dtype=np.uint8)
    dec = np.array([O.b15_decode(int(x)) for x in b], np.float32)
    assert np.array_equal(dec.view(np.uint32), _np_b15_decode(b).view(np.uint32))
    assert all(O.b15_encode(float(d)) == int(x) for d, x in zip(dec, b))  # every byte round-trips
    rng = np.random.default_rng(3)
    f = np.concatenate([rng.uniform(-2.5, 2.5, 4000), rng.uniform(-1e-3, 1e-3, 2000),
                        np.ldexp(1.0, np.arange(-26, 3)).astype(np.float64), [65504.0, 70000.0, -1e30]]).astype(np.float32)
    got = np.array([O.b15_encode(float(x)) for x in f], np.uint8)
    assert np.array_equal(got, _np_b15_encode(f))


def _np_b15_reduce(dt, op, srcs):
    if dt == O.B15:
        a = srcs[0]
        for s in srcs[1:]:
            x, y = _np_b15_decode(a), _np_b15_decode(s)
            r = np.where(x == y, (x.view(np.uint32) | y.view(np.uint32)).view(np.float32), np.fmin(x, y)) \
                if op == O.MIN else x + y
            a = _np_b15_encode(r)
        return a
    if dt == O.B15_ACC_F32:
        a = _np_b15_decode(srcs[0])
        for s in srcs[1:]:
            v = _np_b15_decode(s)
            a = a + v if op == O.SUM else np.where(a < v, a, v)
        return _np_b15_encode(a)
    a = _np_b15_to_h16(srcs[0]).view(np.float16)
    for s in srcs[1:]:
        v = _np_b15_to_h16(s).view(np.float16)
        a = (a + v).astype(np.float16) if op == O.SUM else np.where(a < v, a, v)
    return _np_b15_from_h16(a.view(np.uint16))


@pytest.mark.parametrize("dt", [O.B15, O.B15_ACC_F16, O.B15_ACC_F32, O.U8])
@pytest.mark.parametrize("op", [O.SUM, O.MIN])
@pytest.mark.parametrize("nsrc", [2, 3, 8])
def test_byte_type_reductions_match_numpy(built, dt, op, nsrc):
    rng = np.random.default_rng(100 * dt + 10 * op + nsrc)
    nbytes = 4 * 1024
    srcs = [rng.integers(0, 256, nbytes, dtype=np.uint8) for _ in range(nsrc)]
    got = O.reduce_seq(dt, op, [s.view(np.uint32) for s in srcs]).view(np.uint8)
    if dt == O.U8:
        want = srcs[0].copy()
        for s in srcs[1:]:
            want = (want + s).astype(np.uint8) if op == O.SUM else np.minimum(want, s)
    else:
        want = _np_b15_reduce(dt, op, srcs)
    assert np.array_equal(got, want)
    if nsrc == 2:  # one accumulation step per word, as the kernels' reduce_word
        acc = O.reduce_words(dt, op, srcs[0].view(np.uint32), srcs[1].view(np.uint32)).view(np.uint8)
        assert np.array_equal(acc, want)


def test_b15_order_and_accumulation_matter(built):
    """The three e4m3b15 forms are different reductions (the check is not vacuous): over 8 random
    sources the in-type, half and float accumulations disagree on a share of the bytes."""
    rng = np.random.default_rng(9)
    srcs = [rng.integers(0, 256, 8192, dtype=np.uint8).view(np.uint32) for _ in range(8)]
    r = {dt: O.reduce_seq(dt, O.SUM, srcs).view(np.uint8) for dt in O.B15_TYPES}
    assert (r[O.B15] != r[O.B15_ACC_F32]).mean() > 0.05
    assert (r[O.B15_ACC_F16] != r[O.B15_ACC_F32]).mean() > 0.001
