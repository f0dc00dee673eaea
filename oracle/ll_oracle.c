/*
 * ll_oracle.c -- CPU restatement of microsoft/mscclpp's LL AllReduce hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP path in
 * mscclpp_amd/.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it.  The product library (libmscclpp_amd.so) never links or calls it.
 *
 * Parity pinning: the reference publishes no fp16/bf16 golden sums.  This
 * restatement is pinned by (1) the reference's own known-answer tests (int32 AllReduce
 * input=rank -> n(n-1)/2, test/mscclpp-test/allreduce_test.cu:1172-1183; FIFO fst=snd=i and lap
 * parity, test/unit/fifo_tests.cu:15-153; host-offload AllGather element i = i+1,
 * test/allgather_test_host_offloading.cu:64-79), (2) numpy golden vectors committed under
 * tests/golden/ (tests/golden/make_golden.py), and (3) on the GPU box, by oracle/_ref, a
 * harness that compiles the reference's own device headers (packet_device.hpp,
 * gpu_data_types.hpp) with hipcc and runs them (oracle/build_ref.sh).
 *
 * All citations are path:line under the reference tree (microsoft/mscclpp 0.9.0).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ---- dtype / op codes (mirror include/mscclpp_amd/mscclpp_amd.h) ---------------------- */
enum { ORC_F16 = 0, ORC_BF16 = 1, ORC_F32 = 2, ORC_I32 = 3, ORC_U32 = 4 };
enum { ORC_SUM = 0, ORC_MIN = 1 };

/* ---- scalar conversions ---------------------------------------------------------------- */
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

/* IEEE binary16 -> binary32, exact. */
static float half_to_float(uint16_t h) {
  uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  uint32_t exp = (h >> 10) & 0x1f;
  uint32_t man = h & 0x3ffu;
  if (exp == 0x1f) return u2f(sign | 0x7f800000u | (man << 13)); /* inf / nan (payload kept) */
  if (exp == 0) {
    if (man == 0) return u2f(sign);
    /* subnormal: man * 2^-24 exactly representable in fp32 */
    float v = (float)man * 5.9604644775390625e-08f;
    return (sign ? -v : v);
  }
  return u2f(sign | ((exp + 112u) << 23) | (man << 13));
}

/* binary32 -> binary16 round-to-nearest-even (the rounding of v_cvt_f16_f32 and of the
 * _Float16 add that __hadd2 lowers to, /opt/rocm/include/hip/amd_detail/amd_hip_fp16.h:834). */
static uint16_t float_to_half_rne(float f) {
  uint32_t x = f2u(f);
  uint32_t sign = (x >> 16) & 0x8000u;
  uint32_t absx = x & 0x7fffffffu;
  if (absx >= 0x7f800000u) { /* inf or nan */
    if (absx > 0x7f800000u) return (uint16_t)(sign | 0x7e00u | ((absx >> 13) & 0x3ffu));
    return (uint16_t)(sign | 0x7c00u);
  }
  if (absx >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u); /* >= 65520 rounds to inf */
  if (absx < 0x38800000u) {                                   /* result is subnormal or zero */
    /* value = absx as float; subnormal half = round(value / 2^-24) */
    float a = u2f(absx);
    /* a * 2^24 is exact in fp32 (power of two scale, no overflow) */
    float scaled = a * 16777216.0f;
    /* round half to even on a value < 1024 */
    float fl = floorf(scaled);
    float diff = scaled - fl;
    uint32_t m = (uint32_t)fl;
    if (diff > 0.5f || (diff == 0.5f && (m & 1u))) m++;
    return (uint16_t)(sign | m); /* m may reach 0x400 = smallest normal, still correct */
  }
  /* normal range */
  uint32_t exp = ((absx >> 23) - 112u) << 10;
  uint32_t man = absx & 0x7fffffu;
  uint32_t h = exp | (man >> 13);
  uint32_t rem = man & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
  return (uint16_t)(sign | h);
}

static float bf16_to_float(uint16_t b) { return u2f((uint32_t)b << 16); }

/* binary32 -> bfloat16 RNE (v_cvt_pk_bf16_f32 on gfx950; NaN stays NaN). */
static uint16_t float_to_bf16_rne(float f) {
  uint32_t u = f2u(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

static int half_isnan(uint16_t h) { return (h & 0x7fffu) > 0x7c00u; }
static int bf16_isnan(uint16_t b) { return (b & 0x7fffu) > 0x7f80u; }

/* __hmax/__hmin, /opt/rocm/include/hip/amd_detail/amd_hip_fp16.h:754-775: a NaN operand yields
 * the other operand; both NaN -> canonical NaN; ties return the second (max) / first (min). */
static uint16_t half_max(uint16_t x, uint16_t y) {
  int nx = half_isnan(x), ny = half_isnan(y);
  if (nx && !ny) return y;
  if (!nx && ny) return x;
  if (nx && ny) return 0x7fffu;
  return half_to_float(x) > half_to_float(y) ? x : y;
}
static uint16_t half_min(uint16_t x, uint16_t y) {
  int nx = half_isnan(x), ny = half_isnan(y);
  if (nx && !ny) return y;
  if (!nx && ny) return x;
  if (nx && ny) return 0x7fffu;
  return half_to_float(x) > half_to_float(y) ? y : x;
}
/* bf16 __hmax/__hmin, amd_hip_bf16.h:1295-1315 */
static uint16_t bf16_max(uint16_t a, uint16_t b) {
  int na = bf16_isnan(a), nb = bf16_isnan(b);
  if (na || nb) {
    if (na && nb) return 0x7fffu;
    return na ? b : a;
  }
  return bf16_to_float(a) > bf16_to_float(b) ? a : b;
}
static uint16_t bf16_min(uint16_t a, uint16_t b) {
  int na = bf16_isnan(a), nb = bf16_isnan(b);
  if (na || nb) {
    if (na && nb) return 0x7fffu;
    return na ? b : a;
  }
  return bf16_to_float(a) < bf16_to_float(b) ? a : b;
}

/* clip<__half>, gpu_data_types.hpp:321-326: saturate to [-65504, 65504]; NaN -> -65504. */
static uint16_t half_clip(uint16_t v) { return half_min(half_max(v, 0xfbffu), 0x7bffu); }
/* clip<__bfloat16>, gpu_data_types.hpp:338-342: bounds are -inf/+inf; NaN -> -inf. */
static uint16_t bf16_clip(uint16_t v) { return bf16_min(bf16_max(v, 0xff80u), 0x7f80u); }

/* f16x2 operator+ (gpu_data_types.hpp:389-397): clip(__hadd2(a, b)).  The exact sum of two
 * halves rounded to fp32 then to fp16 equals the correctly rounded fp16 sum (24 >= 2*11+2). */
uint16_t oracle_f16_add(uint16_t a, uint16_t b) {
  return half_clip(float_to_half_rne(half_to_float(a) + half_to_float(b)));
}
/* bf16x2 operator+ (gpu_data_types.hpp:410-418). */
uint16_t oracle_bf16_add(uint16_t a, uint16_t b) {
  return bf16_clip(float_to_bf16_rne(bf16_to_float(a) + bf16_to_float(b)));
}
/* mscclpp::min for f16x2 (gpu_data_types.hpp:605-611) and bf16x2 (:618-620): no clip. */
uint16_t oracle_f16_min(uint16_t a, uint16_t b) { return half_min(a, b); }
uint16_t oracle_bf16_min(uint16_t a, uint16_t b) { return bf16_min(a, b); }
/* f32x2 operator+ (gpu_data_types.hpp:376-387): plain RNE add, no clip. */
uint32_t oracle_f32_add(uint32_t a, uint32_t b) { return f2u(u2f(a) + u2f(b)); }
/* f32x2 min (gpu_data_types.hpp:597-602): fminf. */
uint32_t oracle_f32_min(uint32_t a, uint32_t b) {
  /* llvm.minnum on gfx950 (IEEE mode): a signaling NaN is quieted first, so a NaN operand of
   * either kind yields the other operand; both NaN -> a quiet NaN. */
  int na = (a & 0x7fffffffu) > 0x7f800000u, nb = (b & 0x7fffffffu) > 0x7f800000u;
  if (na && nb) return a | 0x00400000u;
  if (na) return b;
  if (nb) return a;
  return f2u(fminf(u2f(a), u2f(b)));
}

uint16_t oracle_f32_to_f16(float f) { return float_to_half_rne(f); }
uint16_t oracle_f32_to_bf16(float f) { return float_to_bf16_rne(f); }

/* calVectorAccum<T,T,Op> over one 32-bit word (reduce_kernel.hpp:86-134, 171-175). */
static uint32_t reduce_word(int dtype, int op, uint32_t acc, uint32_t val) {
  switch (dtype) {
    case ORC_F16: {
      uint16_t a0 = acc & 0xffff, a1 = acc >> 16, v0 = val & 0xffff, v1 = val >> 16;
      uint16_t r0 = op == ORC_SUM ? oracle_f16_add(a0, v0) : oracle_f16_min(a0, v0);
      uint16_t r1 = op == ORC_SUM ? oracle_f16_add(a1, v1) : oracle_f16_min(a1, v1);
      return (uint32_t)r0 | ((uint32_t)r1 << 16);
    }
    case ORC_BF16: {
      uint16_t a0 = acc & 0xffff, a1 = acc >> 16, v0 = val & 0xffff, v1 = val >> 16;
      uint16_t r0 = op == ORC_SUM ? oracle_bf16_add(a0, v0) : oracle_bf16_min(a0, v0);
      uint16_t r1 = op == ORC_SUM ? oracle_bf16_add(a1, v1) : oracle_bf16_min(a1, v1);
      return (uint32_t)r0 | ((uint32_t)r1 << 16);
    }
    case ORC_F32:
      return op == ORC_SUM ? oracle_f32_add(acc, val) : oracle_f32_min(acc, val);
    case ORC_I32:
      if (op == ORC_SUM) return acc + val; /* wraps, as the device add does */
      return ((int32_t)acc < (int32_t)val) ? acc : val;
    case ORC_U32:
      if (op == ORC_SUM) return acc + val;
      return acc < val ? acc : val;
  }
  return 0;
}

/* acc[i] = acc[i] (op) val[i] for nwords 32-bit words. */
void oracle_reduce_words(int dtype, int op, uint32_t* acc, const uint32_t* val, size_t nwords) {
  for (size_t i = 0; i < nwords; i++) acc[i] = reduce_word(dtype, op, acc[i], val[i]);
}

/* ---- LL packets -------------------------------------------------------------------------- */
/* LL16 packet image {data1, flag1, data2, flag2} (packet_device.hpp:19-48): packet i carries
 * payload words 2i and 2i+1.  copyToPackets<LL16> (copy_device.hpp:156-171). */
void oracle_ll16_pack(const uint32_t* src, size_t npkts, uint32_t flag, uint32_t* pkts) {
  for (size_t i = 0; i < npkts; i++) {
    pkts[4 * i + 0] = src[2 * i];
    pkts[4 * i + 1] = flag;
    pkts[4 * i + 2] = src[2 * i + 1];
    pkts[4 * i + 3] = flag;
  }
}
/* LL16Packet::readOnce (packet_device.hpp:66-82): valid only when both flags equal `flag`.
 * Returns the number of packets whose flags did not match (those words are left untouched). */
size_t oracle_ll16_unpack(const uint32_t* pkts, size_t npkts, uint32_t flag, uint32_t* dst) {
  size_t bad = 0;
  for (size_t i = 0; i < npkts; i++) {
    if (pkts[4 * i + 1] != flag || pkts[4 * i + 3] != flag) { bad++; continue; }
    dst[2 * i] = pkts[4 * i];
    dst[2 * i + 1] = pkts[4 * i + 2];
  }
  return bad;
}
/* LL8 packet image {data, flag} (packet_device.hpp:100-126); copyToPackets<LL8>
 * (copy_device.hpp:173-184). */
void oracle_ll8_pack(const uint32_t* src, size_t npkts, uint32_t flag, uint32_t* pkts) {
  for (size_t i = 0; i < npkts; i++) {
    pkts[2 * i] = src[i];
    pkts[2 * i + 1] = flag;
  }
}
size_t oracle_ll8_unpack(const uint32_t* pkts, size_t npkts, uint32_t flag, uint32_t* dst) {
  size_t bad = 0;
  for (size_t i = 0; i < npkts; i++) {
    if (pkts[2 * i + 1] != flag) { bad++; continue; }
    dst[i] = pkts[2 * i];
  }
  return bad;
}

/* ---- 1-GPU LL16 self-reduce microbench (BASELINE config 2) -----------
 * P = LL16(Y, flag)  [copyToPackets, copy_device.hpp:160-171]
 * O = X (op) unpack(P, flag)  [LL16Packet::read + calVectorAccum, allreduce_packet.cu:93-108]
 * nwords 32-bit words (nwords even).  Returns packets whose flags failed. */
size_t oracle_self_reduce(int dtype, int op, const uint32_t* x, const uint32_t* y, size_t nwords,
                          uint32_t flag, uint32_t* pkts, uint32_t* out) {
  size_t npkts = nwords / 2;
  oracle_ll16_pack(y, npkts, flag, pkts);
  memcpy(out, x, nwords * 4);
  uint32_t* tmp = (uint32_t*)malloc(nwords * 4 + 8);
  size_t bad = oracle_ll16_unpack(pkts, npkts, flag, tmp);
  oracle_reduce_words(dtype, op, out, tmp, nwords);
  free(tmp);
  return bad;
}

/* ---- allreducePacket geometry (allreduce_packet.cu:51-78) ----------- */
typedef struct {
  uint64_t nwords;       /* W: 32-bit words the kernel covers */
  uint64_t npkts;        /* W/2 */
  uint64_t wpr;          /* words per rank slice (made even) */
  uint64_t ppr;          /* packets per rank slice */
  uint64_t in_off;       /* byte offset of peer-input region inside a scratch half: 0 */
  uint64_t result_off;   /* byte offset of reduced-slice region inside a scratch half */
} orc_ll16_geom;

void oracle_ll16_geometry(int dtype, uint64_t count, int n, uint64_t* out6) {
  uint64_t W;
  if (dtype == ORC_F16 || dtype == ORC_BF16)
    W = (count * 2 + 2) / 4; /* :51-52 */
  else
    W = count; /* :53-54, 4-byte types */
  uint64_t wpr = W / (uint64_t)n; /* :62 */
  if (wpr % 2) wpr = wpr + 1;     /* :63, (x*sizeof(T)+sizeof(T))/sizeof(T) = x+1 */
  /* Deviation (documented in DESIGN.md): where the reference's slices stop short of W (W % n != 0
   * with W / n even) its tail words are never reduced; widen by one packet pair in that case only. */
  if (wpr * (uint64_t)n < W) wpr += 2;
  out6[0] = W;
  out6[1] = W / 2;
  out6[2] = wpr;
  out6[3] = wpr / 2;
  out6[4] = 0;
  out6[5] = 2 * (W / 2) * 16; /* scratchResultOffset - base, :74 */
  /* Deviation: keep the reduced-slice region clear of the input-packet region when the slices
   * were rounded up (the reference overlaps them there, a race between ranks). */
  if ((uint64_t)n * (wpr / 2) * 16 > out6[5]) out6[5] = (uint64_t)n * (wpr / 2) * 16;
}

/* Full simulation of one allreducePacket call across n ranks.
 *  in[r]:      rank r's input, padded by the caller to >= n*wpr words (zeros past the data)
 *  scratch[r]: rank r's whole scratch (both halves), half_bytes each; updated in place
 *  out[r]:     rank r's output, >= n*wpr words
 *  Sum order for slice r: x_r first, then peers ascending (:93-106). */
void oracle_allreduce_packet(int dtype, int op, int n, const uint32_t* const* in, uint64_t count,
                             uint32_t flag, uint64_t half_bytes, uint32_t* const* scratch,
                             uint32_t* const* out) {
  uint64_t g[6];
  oracle_ll16_geometry(dtype, count, n, g);
  uint64_t wpr = g[2], ppr = g[3], roff = g[5];
  uint64_t base = (flag % 2) ? half_bytes : 0; /* :60, numScratchBuff = 2 */
  /* step 1: rank s puts its copy of slice q into rank q's scratch at s*ppr packets (:89-90) */
  for (int s = 0; s < n; s++)
    for (int q = 0; q < n; q++) {
      if (q == s) continue;
      uint32_t* dstp = scratch[q] + (base + (uint64_t)s * ppr * 16) / 4;
      oracle_ll16_pack(in[s] + (uint64_t)q * wpr, ppr, flag, dstp);
    }
  /* step 2: rank r reduces its slice and broadcasts reduced packets (:92-123) */
  uint32_t* tmp = (uint32_t*)malloc(wpr * 4 + 8);
  for (int r = 0; r < n; r++) {
    uint32_t* acc = out[r] + (uint64_t)r * wpr;
    memcpy(acc, in[r] + (uint64_t)r * wpr, wpr * 4);
    for (int p = 0; p < n; p++) {
      if (p == r) continue;
      const uint32_t* pk = scratch[r] + (base + (uint64_t)p * ppr * 16) / 4;
      oracle_ll16_unpack(pk, ppr, flag, tmp);
      oracle_reduce_words(dtype, op, acc, tmp, wpr);
    }
    for (int q = 0; q < n; q++) {
      if (q == r) continue;
      uint32_t* dstp = scratch[q] + (base + roff + (uint64_t)r * ppr * 16) / 4;
      oracle_ll16_pack(acc, ppr, flag, dstp);
    }
  }
  /* step 3: unpack the peers' reduced slices (:125-132) */
  for (int r = 0; r < n; r++)
    for (int p = 0; p < n; p++) {
      if (p == r) continue;
      const uint32_t* pk = scratch[r] + (base + roff + (uint64_t)p * ppr * 16) / 4;
      oracle_ll16_unpack(pk, ppr, flag, out[r] + (uint64_t)p * wpr);
    }
  free(tmp);
}

/* allreduceAllPairs (allreduce_allpair_packet.cu:15-69): one-hop LL8.  Rank s writes its
 * whole buffer (W words, W=(2c+2)/4 for 2-byte types) as LL8 packets into every peer's scratch
 * at s*W packets (:28, :40-41); rank r sums x_r then peers ascending (:49-61). */
void oracle_allreduce_allpairs(int dtype, int op, int n, const uint32_t* const* in, uint64_t count,
                               uint32_t flag, uint64_t half_bytes, uint32_t* const* scratch,
                               uint32_t* const* out) {
  uint64_t W = (dtype == ORC_F16 || dtype == ORC_BF16) ? (count * 2 + 2) / 4 : count;
  uint64_t base = (flag % 2) ? half_bytes : 0;
  for (int s = 0; s < n; s++)
    for (int q = 0; q < n; q++) {
      if (q == s) continue;
      oracle_ll8_pack(in[s], W, flag, scratch[q] + (base + (uint64_t)s * W * 8) / 4);
    }
  uint32_t* tmp = (uint32_t*)malloc(W * 4 + 8);
  for (int r = 0; r < n; r++) {
    memcpy(out[r], in[r], W * 4);
    for (int p = 0; p < n; p++) {
      if (p == r) continue;
      oracle_ll8_unpack(scratch[r] + (base + (uint64_t)p * W * 8) / 4, W, flag, tmp);
      oracle_reduce_words(dtype, op, out[r], tmp, W);
    }
  }
  free(tmp);
}

/* Bulk all-pairs result for a word range owned by `owner` with an explicit sum order.
 * order_kind 0: x_owner then peers ascending (allreduce_fullmesh.cu:101-107)
 * order_kind 1: x_owner, x_owner+1, ... mod n (allreduce_rsag.cu:85-94)
 * order_kind 2: ring k1 -- chunk owned by c accumulates from rank c+1 around the ring and the
 *               owner adds last: x_{c+1}, x_{c+2}, ..., x_c (allreduce_test.cu:742-811) */
static void reduce_range(int dtype, int op, int n, const uint32_t* const* in, int owner, int order_kind,
                         uint64_t w0, uint64_t nw, uint32_t* dst) {
  int start = (order_kind == 2) ? (owner + 1) % n : owner;
  memcpy(dst, in[start] + w0, nw * 4);
  if (order_kind == 0) {
    for (int p = 0; p < n; p++)
      if (p != owner) oracle_reduce_words(dtype, op, dst, in[p] + w0, nw);
  } else {
    for (int k = 1; k < n; k++) oracle_reduce_words(dtype, op, dst, in[(start + k) % n] + w0, nw);
  }
}

/* AllReduce over n ranks where slice q (of `slice_words`, the last slice takes the rest) is
 * reduced by rank q in the given order and the result is replicated to every rank.  This is the
 * arithmetic of allreduceFullmesh (kind 0), allreduceRsAg (kind 1) and the k1 ring (kind 2). */
void oracle_allreduce_sliced(int dtype, int op, int n, const uint32_t* const* in, uint64_t nwords,
                             uint64_t slice_words, int order_kind, uint32_t* const* out) {
  for (int q = 0; q < n; q++) {
    uint64_t w0 = (uint64_t)q * slice_words;
    if (w0 >= nwords) break;
    uint64_t nw = (q == n - 1) ? nwords - w0 : slice_words;
    if (w0 + nw > nwords) nw = nwords - w0;
    reduce_range(dtype, op, n, in, q, order_kind, w0, nw, out[0] + w0);
    for (int r = 1; r < n; r++) memcpy(out[r] + w0, out[0] + w0, nw * 4);
  }
}

/* ---- FIFO / ProxyTrigger (fifo_device.hpp:35-141, fifo.cc:58-78) ------------------------- */
void oracle_trigger_encode(uint64_t type, uint32_t dstId, uint64_t dstOffset, uint32_t srcId,
                           uint64_t srcOffset, uint64_t bytes, uint32_t semaphoreId, uint64_t out[2]) {
  const uint64_t m32 = 0xffffffffull, m9 = 0x1ffull, m3 = 0x7ull, m10 = 0x3ffull;
  out[0] = ((srcOffset & m32) << 32) + (bytes & m32); /* :85 */
  out[1] = ((((((((semaphoreId & m10) << 3) + (type & m3)) << 9) + (dstId & m9)) << 9) + (srcId & m9)) << 32) +
           (dstOffset & m32); /* :86-92 */
}
/* Commit bit for slot position pos (fifo_device.hpp:120). */
uint64_t oracle_fifo_commit_bit(uint64_t pos, uint32_t size_shift) { return ((pos >> size_shift) & 1ull) ^ 1ull; }

/* ---- deterministic LCG inputs (test/torch/correctness_test.py:19-22, 44-56) --------------
 * value_i = ((((i + rank + seq) & M) * 1664525 + 1013904223) & M) % 4096 / 4096 as fp32,
 * then cast to the dtype (RNE). */
void oracle_lcg_fill(int dtype, uint64_t count, int rank, int seq, void* dst) {
  for (uint64_t i = 0; i < count; i++) {
    uint64_t s = (i + (uint64_t)rank + (uint64_t)seq) & 0xffffffffull;
    s = (s * 1664525ull + 1013904223ull) & 0xffffffffull;
    float v = (float)(s % 4096) / 4096.0f;
    if (dtype == ORC_F16)
      ((uint16_t*)dst)[i] = float_to_half_rne(v);
    else if (dtype == ORC_BF16)
      ((uint16_t*)dst)[i] = float_to_bf16_rne(v);
    else if (dtype == ORC_F32)
      ((uint32_t*)dst)[i] = f2u(v);
    else
      ((uint32_t*)dst)[i] = (uint32_t)(int32_t)(v * 2147483647.0f);
  }
}
