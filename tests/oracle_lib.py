"""ctypes wrapper around oracle/liboracle.so (the CPU restatement; test infrastructure only)."""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# MSCCLPP_AMD_ORACLE_SO: another build of the same source (the host-sanitizer test loads an ASan/UBSan one)
ORACLE_SO = os.environ.get("MSCCLPP_AMD_ORACLE_SO") or os.path.join(ROOT, "oracle", "liboracle.so")

F16, BF16, F32, I32, U32 = 0, 1, 2, 3, 4
# OCP fp8 reduce types: element type (e4m3 / e5m2) x accumulation type (element, half, float)
E4M3, E5M2, E4M3_ACC_F16, E5M2_ACC_F16, E4M3_ACC_F32, E5M2_ACC_F32 = 5, 6, 7, 8, 9, 10
FP8_TYPES = (E4M3, E5M2, E4M3_ACC_F16, E5M2_ACC_F16, E4M3_ACC_F32, E5M2_ACC_F32)
# uint8 and the software fp8 e4m3b15 accumulated in itself / half / float
U8, B15, B15_ACC_F16, B15_ACC_F32 = 11, 12, 13, 14
B15_TYPES = (B15, B15_ACC_F16, B15_ACC_F32)
BYTE_TYPES = FP8_TYPES + B15_TYPES + (U8,)
SUM, MIN = 0, 1


def itemsize(dtype):
    return 2 if dtype in (F16, BF16) else (1 if dtype in BYTE_TYPES else 4)


def is_e5m2(dtype):
    return dtype in (E5M2, E5M2_ACC_F16, E5M2_ACC_F32)


def ll_words(dtype, count):
    """32-bit words the LL kernels cover (allreduce_packet.cu:51-54 + the 1-byte deviation)."""
    es = itemsize(dtype)
    if es == 4:
        return count
    nbytes = count * es
    w = (nbytes + es) // 4
    return (nbytes + 3) // 4 if w * 4 < nbytes else w

_L = None


def L():
    global _L
    if _L is None:
        if not os.path.exists(ORACLE_SO):
            from mscclpp_amd import _build

            _build.build_oracle()
        _L = ctypes.CDLL(ORACLE_SO)
        u16, u32, u64, sz, vp, i32 = (ctypes.c_uint16, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t,
                                      ctypes.c_void_p, ctypes.c_int)
        for n, a, r in [
            ("oracle_f16_add", [u16, u16], u16), ("oracle_bf16_add", [u16, u16], u16),
            ("oracle_f16_min", [u16, u16], u16), ("oracle_bf16_min", [u16, u16], u16),
            ("oracle_f32_add", [u32, u32], u32), ("oracle_f32_min", [u32, u32], u32),
            ("oracle_reduce_words", [i32, i32, vp, vp, sz], None),
            ("oracle_reduce_seq", [i32, i32, i32, vp, sz, vp], None),
            ("oracle_fp8_encode_sat", [ctypes.c_float, i32], ctypes.c_uint8),
            ("oracle_fp8_decode", [ctypes.c_uint8, i32], ctypes.c_float),
            ("oracle_b15_encode", [ctypes.c_float], ctypes.c_uint8),
            ("oracle_b15_decode", [ctypes.c_uint8], ctypes.c_float),
            ("oracle_ll16_pack", [vp, sz, u32, vp], None), ("oracle_ll16_unpack", [vp, sz, u32, vp], sz),
            ("oracle_ll8_pack", [vp, sz, u32, vp], None), ("oracle_ll8_unpack", [vp, sz, u32, vp], sz),
            ("oracle_self_reduce", [i32, i32, vp, vp, sz, u32, vp, vp], sz),
            ("oracle_ll16_geometry", [i32, u64, i32, vp], None),
            ("oracle_allreduce_packet", [i32, i32, i32, vp, u64, u32, u64, vp, vp], None),
            ("oracle_allreduce_allpairs", [i32, i32, i32, vp, u64, u32, u64, vp, vp], None),
            ("oracle_allreduce_sliced", [i32, i32, i32, vp, u64, u64, i32, vp], None),
            ("oracle_mscclpp_test_ll", [i32, vp, u64, u32, vp, vp], None),
            ("oracle_bench_allreduce2", [i32, i32, i32, vp, u64, u32, vp, vp], None),
            ("oracle_bench_allreduce1", [i32, i32, vp, u64, vp], None),
            ("oracle_mscclpp_test_k2", [i32, vp, u64, u32, vp, vp], None),
            ("oracle_allreduce_owned", [i32, i32, i32, vp, u64, u64, u64, i32, vp], None),
            ("oracle_trigger_encode", [u64, u32, u64, u32, u64, u64, u32, vp], None),
            ("oracle_fifo_commit_bit", [u64, u32], u64),
            ("oracle_lcg_fill", [i32, u64, i32, i32, vp], None),
        ]:
            f = getattr(_L, n)
            f.argtypes = a
            f.restype = r
    return _L


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _ptr_array(arrs):
    t = (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    return t


def reduce_words(dtype, op, acc, val):
    acc = np.ascontiguousarray(acc, dtype=np.uint32).copy()
    val = np.ascontiguousarray(val, dtype=np.uint32)
    L().oracle_reduce_words(dtype, op, _p(acc), _p(val), acc.size)
    return acc


def ll16_pack(words, flag):
    words = np.ascontiguousarray(words, dtype=np.uint32)
    out = np.zeros(words.size * 2, np.uint32)
    L().oracle_ll16_pack(_p(words), words.size // 2, flag, _p(out))
    return out


def ll8_pack(words, flag):
    words = np.ascontiguousarray(words, dtype=np.uint32)
    out = np.zeros(words.size * 2, np.uint32)
    L().oracle_ll8_pack(_p(words), words.size, flag, _p(out))
    return out


def self_reduce(dtype, op, x, y, flag):
    x = np.ascontiguousarray(x).view(np.uint32)
    y = np.ascontiguousarray(y).view(np.uint32)
    pk = np.zeros(x.size * 2, np.uint32)
    out = np.zeros(x.size, np.uint32)
    bad = L().oracle_self_reduce(dtype, op, _p(x), _p(y), x.size, flag, _p(pk), _p(out))
    assert bad == 0
    return pk, out


def geometry(dtype, count, n):
    g = np.zeros(6, np.uint64)
    L().oracle_ll16_geometry(dtype, count, n, _p(g))
    return [int(v) for v in g]


def allreduce_packet(dtype, op, inputs, count, flag, half_bytes):
    n = len(inputs)
    W, npk, wpr, ppr, _, roff = geometry(dtype, count, n)
    nw = max(W, n * wpr)
    ins = [np.zeros(nw + 4, np.uint32) for _ in range(n)]
    for r in range(n):
        src = np.ascontiguousarray(inputs[r]).view(np.uint8)
        ins[r].view(np.uint8)[: src.size] = src
    scr = [np.zeros(2 * half_bytes // 4, np.uint32) for _ in range(n)]
    outs = [np.zeros(nw + 4, np.uint32) for _ in range(n)]
    L().oracle_allreduce_packet(dtype, op, n, _ptr_array(ins), count, flag, half_bytes, _ptr_array(scr),
                                _ptr_array(outs))
    return outs, scr


def allreduce_allpairs(dtype, op, inputs, count, flag, half_bytes):
    n = len(inputs)
    W = ll_words(dtype, count)
    ins = [np.zeros(W + 4, np.uint32) for _ in range(n)]
    for r in range(n):
        src = np.ascontiguousarray(inputs[r]).view(np.uint8)
        ins[r].view(np.uint8)[: src.size] = src
    scr = [np.zeros(2 * half_bytes // 4, np.uint32) for _ in range(n)]
    outs = [np.zeros(W + 4, np.uint32) for _ in range(n)]
    L().oracle_allreduce_allpairs(dtype, op, n, _ptr_array(ins), count, flag, half_bytes, _ptr_array(scr),
                                  _ptr_array(outs))
    return outs, scr


def mscclpp_test_ll(inputs, nelems, flag, scratch_bytes):
    """mscclpp-test allreduce6/7: outputs and the full scratch images (harness layout)."""
    n = len(inputs)
    ins = [np.ascontiguousarray(a).view(np.uint32) for a in inputs]
    scr = [np.zeros(scratch_bytes // 4, np.uint32) for _ in range(n)]
    outs = [np.zeros(nelems, np.uint32) for _ in range(n)]
    L().oracle_mscclpp_test_ll(n, _ptr_array(ins), nelems, flag, _ptr_array(scr), _ptr_array(outs))
    return outs, scr


def bench_allreduce2(dtype, inputs, nwords, flag, scratch_bytes, order=0):
    """python/mscclpp_benchmark/allreduce.cu allreduce2 with TYPE = int (I32), float (F32) or __half
    (F16): outputs and full scratch images.  order 0 is the kernel's (0 + peers ascending + own);
    order 1 (own + peers ascending) exists only to show that a test tells the two apart."""
    n = len(inputs)
    ins = [np.ascontiguousarray(a).view(np.uint32) for a in inputs]
    scr = [np.zeros(scratch_bytes // 4, np.uint32) for _ in range(n)]
    outs = [np.zeros(nwords, np.uint32) for _ in range(n)]
    L().oracle_bench_allreduce2(dtype, order, n, _ptr_array(ins), nwords, flag, _ptr_array(scr), _ptr_array(outs))
    return outs, scr


def bench_allreduce1(dtype, inputs, nwords):
    """python/mscclpp_benchmark/allreduce.cu allreduce1 (in place, own chunk first then the peers in
    the kernel's rotated channel order): every rank's resulting buffer."""
    n = len(inputs)
    ins = [np.ascontiguousarray(a).view(np.uint32) for a in inputs]
    outs = [np.zeros(nwords, np.uint32) for _ in range(n)]
    L().oracle_bench_allreduce1(dtype, n, _ptr_array(ins), nwords, _ptr_array(outs))
    return outs


def mscclpp_test_k2(inputs, nelems, flag, scratch_bytes):
    """mscclpp-test allreduce2 on one node: outputs and the full scratch images (harness layout)."""
    n = len(inputs)
    ins = [np.ascontiguousarray(a).view(np.uint32) for a in inputs]
    scr = [np.zeros(scratch_bytes // 4, np.uint32) for _ in range(n)]
    outs = [np.zeros(nelems, np.uint32) for _ in range(n)]
    L().oracle_mscclpp_test_k2(n, _ptr_array(ins), nelems, flag, _ptr_array(scr), _ptr_array(outs))
    return outs, scr


def allreduce_sliced(dtype, op, inputs, nwords, slice_words, order_kind):
    n = len(inputs)
    ins = [np.ascontiguousarray(a).view(np.uint32) for a in inputs]
    outs = [np.zeros(nwords, np.uint32) for _ in range(n)]
    L().oracle_allreduce_sliced(dtype, op, n, _ptr_array(ins), nwords, slice_words, order_kind, _ptr_array(outs))
    return outs


def allreduce_owned(dtype, op, inputs, nwords, period_words, chunk_words, order_kind):
    """One AllReduce result buffer: word w owned by (w % period) // chunk, reduced in that owner's
    order (0 fullmesh: owner then ascending; 1 ring: owner, owner+1, ...)."""
    n = len(inputs)
    ins = []
    for a in inputs:
        w = np.ascontiguousarray(a).view(np.uint8)
        if w.size < nwords * 4:  # pad a ragged tail with zeros (the kernels' 16-byte units)
            p = np.zeros(nwords * 4, np.uint8)
            p[: w.size] = w
            w = p
        ins.append(w.view(np.uint32))
    out = np.zeros(nwords, np.uint32)
    L().oracle_allreduce_owned(dtype, op, n, _ptr_array(ins), nwords, period_words, chunk_words, order_kind, _p(out))
    return out


def trigger_encode(typ, dst_id, dst_off, src_id, src_off, nbytes, sem):
    out = np.zeros(2, np.uint64)
    L().oracle_trigger_encode(typ, dst_id, dst_off, src_id, src_off, nbytes, sem, _p(out))
    return int(out[0]), int(out[1])


def lcg(dtype, count, rank, seq):
    isz = itemsize(dtype)
    out = np.zeros(count * isz, np.uint8)
    L().oracle_lcg_fill(dtype, count, rank, seq, _p(out))
    return out.view({1: np.uint8, 2: np.uint16, 4: np.uint32}[isz])


def reduce_seq(dtype, op, srcs):
    """srcs[0] (op) srcs[1] (op) ... in order, accumulated in the reduce type's AccumT."""
    srcs = [np.ascontiguousarray(a).view(np.uint32) for a in srcs]
    out = np.zeros(srcs[0].size, np.uint32)
    L().oracle_reduce_seq(dtype, op, len(srcs), _ptr_array(srcs), out.size, _p(out))
    return out


def fp8_decode(b, e5m2):
    return L().oracle_fp8_decode(int(b), int(e5m2))


def fp8_encode_sat(f, e5m2):
    return int(L().oracle_fp8_encode_sat(float(f), int(e5m2)))


def b15_encode(f):
    return int(L().oracle_b15_encode(float(f)))


def b15_decode(b):
    return L().oracle_b15_decode(int(b))
