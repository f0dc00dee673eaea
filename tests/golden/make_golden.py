"""Generate the golden fixtures in tests/golden/golden_v1.npz with numpy only.

This script is independent of oracle/ll_oracle.c: it restates the same reference semantics
with numpy so the C oracle can be pinned against it (tests/test_oracle_golden.py).  It never
imports or runs anything from the reference tree; the reference is only cited:

* fp16 add = clip(__hadd2(a, b))                  include/mscclpp/gpu_data_types.hpp:389-397, 321-326
* bf16 add = clip(__hadd2(a, b)), bounds +-inf    include/mscclpp/gpu_data_types.hpp:410-418, 338-342
* __hmax/__hmin NaN rules                         /opt/rocm/include/hip/amd_detail/amd_hip_fp16.h:754-775
* LL16 / LL8 packet images                         include/mscclpp/packet_device.hpp:19-159
* allreducePacket geometry and sum order          src/ext/collectives/allreduce/allreduce_packet.cu:51-140
* allreduceAllPairs                               src/ext/collectives/allreduce/allreduce_allpair_packet.cu:15-69
* fullmesh / rsag / k1-ring sum orders            allreduce_fullmesh.cu:101-107, allreduce_rsag.cu:85-94,
                                                  test/mscclpp-test/allreduce_test.cu:742-811
* LCG inputs                                      test/torch/correctness_test.py:19-22, 44-56
* int32 KAT input=rank -> n(n-1)/2                test/mscclpp-test/allreduce_test.cu:1172-1183
* ProxyTrigger bit layout                         include/mscclpp/fifo_device.hpp:35-92

Run:  python tests/golden/make_golden.py   (writes golden_v1.npz next to this file and
prints its sha256, recorded in tests/golden/MANIFEST.txt)
"""
import hashlib
import os

import numpy as np

F16, BF16, F32, I32 = 0, 1, 2, 3
SUM, MIN = 0, 1

# ---------------------------------------------------------------- scalar arithmetic


def f16_bits(x):
    return np.asarray(x, dtype=np.float16).view(np.uint16)


def f16_from_bits(b):
    return np.asarray(b, dtype=np.uint16).view(np.float16)


def bf16_to_f32(b):
    return (np.asarray(b, dtype=np.uint32) << 16).view(np.float32)


def f32_to_bf16(f):
    u = np.asarray(f, dtype=np.float32).view(np.uint32).astype(np.uint64)
    nan = (u & 0x7FFFFFFF) > 0x7F800000
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    return np.where(nan, ((u >> 16) | 0x40).astype(np.uint16), r)


def _nan16(b):
    return (b & 0x7FFF) > 0x7C00


def _nanbf(b):
    return (b & 0x7FFF) > 0x7F80


def hmax16(x, y):
    fx, fy = f16_from_bits(x).astype(np.float32), f16_from_bits(y).astype(np.float32)
    nx, ny = _nan16(x), _nan16(y)
    r = np.where(fx > fy, x, y)
    r = np.where(nx & ~ny, y, r)
    r = np.where(~nx & ny, x, r)
    return np.where(nx & ny, np.uint16(0x7FFF), r).astype(np.uint16)


def hmin16(x, y):
    fx, fy = f16_from_bits(x).astype(np.float32), f16_from_bits(y).astype(np.float32)
    nx, ny = _nan16(x), _nan16(y)
    r = np.where(fx > fy, y, x)
    r = np.where(nx & ~ny, y, r)
    r = np.where(~nx & ny, x, r)
    return np.where(nx & ny, np.uint16(0x7FFF), r).astype(np.uint16)


def hmaxbf(a, b):
    fa, fb = bf16_to_f32(a), bf16_to_f32(b)
    na, nb = _nanbf(a), _nanbf(b)
    r = np.where(fa > fb, a, b)
    r = np.where(na & ~nb, b, r)
    r = np.where(~na & nb, a, r)
    return np.where(na & nb, np.uint16(0x7FFF), r).astype(np.uint16)


def hminbf(a, b):
    fa, fb = bf16_to_f32(a), bf16_to_f32(b)
    na, nb = _nanbf(a), _nanbf(b)
    r = np.where(fa < fb, a, b)
    r = np.where(na & ~nb, b, r)
    r = np.where(~na & nb, a, r)
    return np.where(na & nb, np.uint16(0x7FFF), r).astype(np.uint16)


def add16(a, b):
    with np.errstate(all="ignore"):
        s = f16_bits(f16_from_bits(a) + f16_from_bits(b))
    return hmin16(hmax16(s, np.uint16(0xFBFF)), np.uint16(0x7BFF))


def addbf(a, b):
    with np.errstate(all="ignore"):
        s = f32_to_bf16(bf16_to_f32(a) + bf16_to_f32(b))
    return hminbf(hmaxbf(s, np.uint16(0xFF80)), np.uint16(0x7F80))


def add32(a, b):
    with np.errstate(all="ignore"):
        return (np.asarray(a, np.uint32).view(np.float32) + np.asarray(b, np.uint32).view(np.float32)).view(np.uint32)


def min32(a, b):
    with np.errstate(all="ignore"):
        return np.fmin(np.asarray(a, np.uint32).view(np.float32), np.asarray(b, np.uint32).view(np.float32)).view(
            np.uint32
        )


def reduce_words(dtype, op, acc, val):
    """acc, val: uint32 word arrays -> uint32 words."""
    acc = np.asarray(acc, np.uint32)
    val = np.asarray(val, np.uint32)
    if dtype in (F16, BF16):
        a16, v16 = acc.view(np.uint16), val.view(np.uint16)
        if dtype == F16:
            r = add16(a16, v16) if op == SUM else hmin16(a16, v16)
        else:
            r = addbf(a16, v16) if op == SUM else hminbf(a16, v16)
        return np.ascontiguousarray(r).view(np.uint32)
    if dtype == F32:
        return add32(acc, val) if op == SUM else min32(acc, val)
    if op == SUM:
        return (acc.astype(np.uint64) + val.astype(np.uint64)).astype(np.uint32)
    return np.where(acc.view(np.int32) < val.view(np.int32), acc, val).astype(np.uint32)


# ---------------------------------------------------------------- packets


def ll16_pack(words, flag):
    n = words.size // 2
    p = np.empty((n, 4), np.uint32)
    p[:, 0] = words[0::2][:n]
    p[:, 1] = flag
    p[:, 2] = words[1::2][:n]
    p[:, 3] = flag
    return p.reshape(-1)


def ll8_pack(words, flag):
    p = np.empty((words.size, 2), np.uint32)
    p[:, 0] = words
    p[:, 1] = flag
    return p.reshape(-1)


def ll16_unpack(pk):
    p = pk.reshape(-1, 4)
    out = np.empty(p.shape[0] * 2, np.uint32)
    out[0::2] = p[:, 0]
    out[1::2] = p[:, 2]
    return out


def ll8_unpack(pk):
    return pk.reshape(-1, 2)[:, 0].copy()


# ---------------------------------------------------------------- inputs


def lcg(dtype, count, rank, seq):
    i = np.arange(count, dtype=np.uint64)
    s = (i + rank + seq) & 0xFFFFFFFF
    s = (s * 1664525 + 1013904223) & 0xFFFFFFFF
    base = (s % 4096).astype(np.float32) / np.float32(4096.0)
    if dtype == F16:
        return base.astype(np.float16).view(np.uint16)
    if dtype == BF16:
        return f32_to_bf16(base)
    if dtype == F32:
        return base.view(np.uint32)
    return (base * np.float32(2**31 - 1)).astype(np.int32).view(np.uint32)


def to_words(arr, nwords):
    b = np.zeros(nwords * 4, np.uint8)
    raw = np.ascontiguousarray(arr).view(np.uint8)
    b[: min(raw.size, b.size)] = raw[: b.size]
    return b.view(np.uint32)


# ---------------------------------------------------------------- collectives


def geometry(dtype, count, n):
    W = (count * 2 + 2) // 4 if dtype in (F16, BF16) else count
    wpr = W // n
    if wpr % 2:
        wpr += 1
    if wpr * n < W:  # mscclpp_amd deviation: the reference would leave the tail unreduced
        wpr += 2
    roff = max(2 * (W // 2) * 16, n * (wpr // 2) * 16)  # deviation: no input/result overlap
    return W, W // 2, wpr, wpr // 2, roff


def allreduce_packet(dtype, op, inputs_words, count, flag, half_bytes):
    n = len(inputs_words)
    W, npk, wpr, ppr, roff = geometry(dtype, count, n)
    base = half_bytes if flag % 2 else 0
    scratch = [np.zeros(2 * half_bytes // 4, np.uint32) for _ in range(n)]
    out = [np.zeros(n * wpr, np.uint32) for _ in range(n)]
    for s in range(n):
        for q in range(n):
            if q != s:
                o = (base + s * ppr * 16) // 4
                scratch[q][o : o + ppr * 4] = ll16_pack(inputs_words[s][q * wpr : (q + 1) * wpr], flag)
    for r in range(n):
        acc = inputs_words[r][r * wpr : (r + 1) * wpr].copy()
        for p in range(n):
            if p != r:
                o = (base + p * ppr * 16) // 4
                acc = reduce_words(dtype, op, acc, ll16_unpack(scratch[r][o : o + ppr * 4]))
        out[r][r * wpr : (r + 1) * wpr] = acc
        for q in range(n):
            if q != r:
                o = (base + roff + r * ppr * 16) // 4
                scratch[q][o : o + ppr * 4] = ll16_pack(acc, flag)
    for r in range(n):
        for p in range(n):
            if p != r:
                o = (base + roff + p * ppr * 16) // 4
                out[r][p * wpr : (p + 1) * wpr] = ll16_unpack(scratch[r][o : o + ppr * 4])
    return out, scratch


def allreduce_allpairs(dtype, op, inputs_words, count, flag, half_bytes):
    n = len(inputs_words)
    W = (count * 2 + 2) // 4 if dtype in (F16, BF16) else count
    base = half_bytes if flag % 2 else 0
    scratch = [np.zeros(2 * half_bytes // 4, np.uint32) for _ in range(n)]
    for s in range(n):
        for q in range(n):
            if q != s:
                o = (base + s * W * 8) // 4
                scratch[q][o : o + 2 * W] = ll8_pack(inputs_words[s][:W], flag)
    out = []
    for r in range(n):
        acc = inputs_words[r][:W].copy()
        for p in range(n):
            if p != r:
                o = (base + p * W * 8) // 4
                acc = reduce_words(dtype, op, acc, ll8_unpack(scratch[r][o : o + 2 * W]))
        out.append(acc)
    return out, scratch


def allreduce_sliced(dtype, op, inputs_words, nwords, slice_words, order_kind):
    n = len(inputs_words)
    res = np.zeros(nwords, np.uint32)
    for q in range(n):
        w0 = q * slice_words
        if w0 >= nwords:
            break
        nw = nwords - w0 if q == n - 1 else min(slice_words, nwords - w0)
        if order_kind == 0:
            order = [q] + [p for p in range(n) if p != q]
        elif order_kind == 1:
            order = [(q + k) % n for k in range(n)]
        else:
            order = [(q + 1 + k) % n for k in range(n)]
        acc = inputs_words[order[0]][w0 : w0 + nw].copy()
        for p in order[1:]:
            acc = reduce_words(dtype, op, acc, inputs_words[p][w0 : w0 + nw])
        res[w0 : w0 + nw] = acc
    return res


def trigger_encode(typ, dst_id, dst_off, src_id, src_off, nbytes, sem_id):
    fst = ((src_off & 0xFFFFFFFF) << 32) + (nbytes & 0xFFFFFFFF)
    snd = ((((((((sem_id & 0x3FF) << 3) + (typ & 7)) << 9) + (dst_id & 0x1FF)) << 9) + (src_id & 0x1FF)) << 32) + (
        dst_off & 0xFFFFFFFF
    )
    return fst & 0xFFFFFFFFFFFFFFFF, snd & 0xFFFFFFFFFFFFFFFF


# ---------------------------------------------------------------- fixture assembly

SPECIAL16 = [0x0000, 0x8000, 0x3C00, 0xBC00, 0x7BFF, 0xFBFF, 0x7BFE, 0x7C00, 0xFC00, 0x7E00, 0x7C01, 0xFE00,
             0x0001, 0x8001, 0x03FF, 0x0400, 0x8400, 0x3555, 0x5BFF, 0x7800, 0xF800, 0x1000, 0x2E66, 0x6400]
SPECIALBF = [0x0000, 0x8000, 0x3F80, 0xBF80, 0x7F7F, 0xFF7F, 0x7F80, 0xFF80, 0x7FC0, 0x7F81, 0xFFC0,
             0x0001, 0x8001, 0x007F, 0x0080, 0x8080, 0x3EAB, 0x4B00, 0x7F00, 0xFF00, 0x3DCD]
SPECIAL32 = [0x00000000, 0x80000000, 0x3F800000, 0xBF800000, 0x7F7FFFFF, 0xFF7FFFFF, 0x7F800000, 0xFF800000,
             0x00000001, 0x80000001, 0x007FFFFF, 0x00800000, 0x33800000, 0x4B800000, 0x3DCCCCCD]


def pairs(special, rng, bits, nrand):
    s = np.array(special, dtype=np.uint64)
    a, b = np.meshgrid(s, s, indexing="ij")
    a, b = a.reshape(-1), b.reshape(-1)
    ra = rng.integers(0, 2**bits, nrand, dtype=np.uint64)
    rb = rng.integers(0, 2**bits, nrand, dtype=np.uint64)
    dt = np.uint16 if bits == 16 else np.uint32
    return np.concatenate([a, ra]).astype(dt), np.concatenate([b, rb]).astype(dt)


def main():
    rng = np.random.default_rng(20260821)
    g = {}
    a, b = pairs(SPECIAL16, rng, 16, 8192)
    g["f16_a"], g["f16_b"], g["f16_add"], g["f16_min"] = a, b, add16(a, b), hmin16(a, b)
    a, b = pairs(SPECIALBF, rng, 16, 8192)
    g["bf16_a"], g["bf16_b"], g["bf16_add"], g["bf16_min"] = a, b, addbf(a, b), hminbf(a, b)
    a, b = pairs(SPECIAL32, rng, 32, 8192)
    g["f32_a"], g["f32_b"], g["f32_add"], g["f32_min"] = a, b, add32(a, b), min32(a, b)
    # LCG inputs
    g["lcg_f16_r3_s1"] = lcg(F16, 1000, 3, 1)
    g["lcg_bf16_r3_s1"] = lcg(BF16, 1000, 3, 1)
    g["lcg_f32_r3_s1"] = lcg(F32, 1000, 3, 1)
    # packets
    w = rng.integers(0, 2**32, 64, dtype=np.uint64).astype(np.uint32)
    g["pkt_words"] = w
    g["pkt_ll16_flag7"] = ll16_pack(w, 7)
    g["pkt_ll8_flag7"] = ll8_pack(w, 7)
    # self-reduce microbench: x, y fp16 LCG ranks 0/1 seq 0, flag 1
    x, y = lcg(F16, 4096, 0, 0), lcg(F16, 4096, 1, 0)
    xw, yw = to_words(x, 2048), to_words(y, 2048)
    g["self_x"], g["self_y"] = xw, yw
    g["self_pkts"] = ll16_pack(yw, 1)
    g["self_out"] = reduce_words(F16, SUM, xw, yw)
    # collectives: (algorithm, n, dtype, count, flag)
    half_bytes = 1 << 16
    cases = []
    for n in (2, 4, 8):
        for dt, count in ((F16, 2048), (BF16, 2048), (F32, 1024), (I32, 1024)):
            cases.append(("packet", n, dt, count, 1 if n != 4 else 2))
            cases.append(("allpairs", n, dt, count // 4, 1))
    for key, (algo, n, dt, count, flag) in enumerate(cases):
        W = (count * 2 + 2) // 4 if dt in (F16, BF16) else count
        _, _, wpr, _, _ = geometry(dt, count, n)
        nw = max(W, n * wpr)
        ins = [to_words(lcg(dt, count, r, 0), nw) for r in range(n)]
        if algo == "packet":
            outs, scr = allreduce_packet(dt, SUM, ins, count, flag, half_bytes)
        else:
            outs, scr = allreduce_allpairs(dt, SUM, ins, count, flag, half_bytes)
        pref = f"coll{key}_"
        g[pref + "meta"] = np.array([0 if algo == "packet" else 1, n, dt, count, flag, half_bytes], np.int64)
        g[pref + "in"] = np.stack(ins)
        g[pref + "out"] = np.stack([o[:W] for o in outs])
        g[pref + "scratch"] = np.stack(scr)
    # bulk orders (fullmesh / rsag / ring) for fp32 and fp16, n = 8
    for kind in (0, 1, 2):
        for dt in (F32, F16):
            nwords = 8 * 96
            ins = [lcg(dt, nwords * (2 if dt == F16 else 1), r, 5).view(np.uint32) for r in range(8)]
            g[f"bulk{kind}_{dt}_in"] = np.stack(ins)
            g[f"bulk{kind}_{dt}_out"] = allreduce_sliced(dt, SUM, ins, nwords, 96, kind)
    # int32 KAT (allreduce_test.cu:1172-1183)
    g["kat_i32_n8"] = np.full(256, 8 * 7 // 2, np.int32)
    # triggers
    trig = []
    for i in range(64):
        vals = [int(v) for v in rng.integers(0, 2**31, 7)]
        typ, dst_id, dst_off, src_id, src_off, nbytes, sem = (vals[0] % 8, vals[1] % 512, vals[2], vals[3] % 512,
                                                              vals[4], vals[5], vals[6] % 1024)
        fst, snd = trigger_encode(typ, dst_id, dst_off, src_id, src_off, nbytes, sem)
        trig.append([typ, dst_id, dst_off, src_id, src_off, nbytes, sem, fst, snd])
    g["triggers"] = np.array(trig, dtype=np.uint64)
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden_v1.npz")
    np.savez_compressed(out, **g)
    h = hashlib.sha256(open(out, "rb").read()).hexdigest()
    print(out, h)


if __name__ == "__main__":
    main()
