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
/* OCP FP8 reduce types: element e4m3 / e5m2, accumulated in the element type, half or float
 * (calVectorAccum<T, AccumT>, src/core/include/reduce_kernel.hpp:139-189; common.hpp:89-100). */
enum { ORC_E4M3 = 5, ORC_E5M2 = 6, ORC_E4M3_ACC_F16 = 7, ORC_E5M2_ACC_F16 = 8, ORC_E4M3_ACC_F32 = 9,
       ORC_E5M2_ACC_F32 = 10 };
/* uint8 (Adapter<Op, uint8_t, uint8_t>, common.hpp:132-133) and the software fp8 e4m3b15
 * accumulated in itself, half or float (dispatchFp8Accum, common.hpp:89-100, :128-129). */
enum { ORC_U8 = 11, ORC_B15 = 12, ORC_B15_ACC_F16 = 13, ORC_B15_ACC_F32 = 14 };
enum { ORC_SUM = 0, ORC_MIN = 1 };

static int orc_is_fp8(int dt) { return dt >= ORC_E4M3 && dt <= ORC_E5M2_ACC_F32; }
static int orc_is_b15(int dt) { return dt >= ORC_B15 && dt <= ORC_B15_ACC_F32; }
static int orc_is_byte(int dt) { return orc_is_fp8(dt) || orc_is_b15(dt) || dt == ORC_U8; }
static int orc_is_e5m2(int dt) { return dt == ORC_E5M2 || dt == ORC_E5M2_ACC_F16 || dt == ORC_E5M2_ACC_F32; }
static int orc_acc_kind(int dt) {
  if (dt == ORC_E4M3_ACC_F16 || dt == ORC_E5M2_ACC_F16 || dt == ORC_B15_ACC_F16) return 1;
  if (dt == ORC_E4M3_ACC_F32 || dt == ORC_E5M2_ACC_F32 || dt == ORC_B15_ACC_F32) return 2;
  return 0;
}
static int orc_elem_bytes(int dt) { return (dt == ORC_F16 || dt == ORC_BF16) ? 2 : (orc_is_byte(dt) ? 1 : 4); }

/* 32-bit words the LL kernels cover: (count*sizeof(T)+sizeof(T))/4 for 1- and 2-byte T
 * (allreduce_packet.cu:51-54, allreduce_allpair_packet.cu:20).  Deviation: 1-byte T
 * with count % 4 in {1, 2} would stop short of the buffer, so W is rounded up there only. */
static uint64_t orc_ll_words(int dt, uint64_t count) {
  int es = orc_elem_bytes(dt);
  uint64_t bytes = count * (uint64_t)es;
  if (es == 4) return count;
  uint64_t W = (bytes + (uint64_t)es) / 4;
  if (W * 4 < bytes) W = (bytes + 3) / 4;
  return W;
}

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
  if (u2f(a) == u2f(b)) return a | b; /* v_min_f32 orders -0 below +0 */
  return f2u(fminf(u2f(a), u2f(b)));
}

uint16_t oracle_f32_to_f16(float f) { return float_to_half_rne(f); }
uint16_t oracle_f32_to_bf16(float f) { return float_to_bf16_rne(f); }

/* ---- OCP FP8 (gfx950 formats) ---------------------------------------------------------------
 * The reference's ROCm gfx950 build takes the generic branches of gpu_data_types.hpp (the packed
 * fp8 paths there are gfx942-only), so per element:
 *   float(fp8)        -> v_cvt_f32_fp8 / _bf8: exact for finite values        (amd_hip_fp8.h:638-650)
 *   __hip_fp8_*(f)    -> non-NaN/Inf saturated to +-448 / +-57344, then RNE  (amd_hip_fp8.h:548-592)
 * The NaN / Inf images of the two hardware conversions were pinned against the device by
 * tests/test_fp8_gpu.py (the reference's own conversions run on the GPU): every NaN byte decodes
 * to 0xFFC00000; every float NaN encodes to 0xFF (e4m3) / 0xFE (e5m2); +-Inf encodes to 0x7F/0xFF
 * (e4m3, no infinities) and 0x7C/0xFC (e5m2). */
static float fp8_decode(uint8_t b, int e5m2) {
  uint32_t sign = (b & 0x80u) ? 0x80000000u : 0u;
  float v;
  if (!e5m2) {
    uint32_t e = (b >> 3) & 0xfu, m = b & 7u;
    if ((b & 0x7fu) == 0x7fu) return u2f(0xffc00000u);
    v = e ? ldexpf(1.0f + (float)m / 8.0f, (int)e - 7) : ldexpf((float)m / 8.0f, -6);
  } else {
    uint32_t e = (b >> 2) & 0x1fu, m = b & 3u;
    if (e == 0x1fu) return m ? u2f(0xffc00000u) : u2f(sign | 0x7f800000u);
    v = e ? ldexpf(1.0f + (float)m / 4.0f, (int)e - 15) : ldexpf((float)m / 4.0f, -14);
  }
  return sign ? -v : v;
}

/* hardware float -> fp8 (no clamp), RNE; NaN / Inf images as the device produces them */
static uint8_t fp8_encode_hw(float f, int e5m2) {
  uint32_t x = f2u(f);
  uint8_t sign = (uint8_t)((x >> 24) & 0x80u);
  float a = fabsf(f);
  if ((x & 0x7fffffffu) > 0x7f800000u) return e5m2 ? 0xfeu : 0xffu;            /* NaN, any sign */
  if ((x & 0x7fffffffu) == 0x7f800000u) return (uint8_t)(sign | (e5m2 ? 0x7cu : 0x7fu)); /* Inf */
  int mbits = e5m2 ? 2 : 3, bias = e5m2 ? 15 : 7;
  int emin = 1 - bias; /* smallest normal exponent */
  if (a < ldexpf(1.0f, emin)) {
    /* subnormal range: integer multiple of 2^(emin - mbits); a carry to 2^mbits is the smallest normal */
    float q = rintf(ldexpf(a, mbits - emin));
    return (uint8_t)(sign | (uint8_t)q);
  }
  int e;
  frexpf(a, &e); /* a = fr * 2^e, fr in [0.5, 1) */
  e -= 1;        /* a = 1.m * 2^e */
  float r = rintf(ldexpf(a, mbits - e)); /* in [2^mbits, 2^(mbits+1)] */
  uint32_t bits = ((uint32_t)(e + bias) << mbits) + (uint32_t)r - (1u << mbits);
  uint32_t maxbits = e5m2 ? 0x7bu : 0x7eu;
  if (bits > maxbits) bits = e5m2 ? 0x7cu : 0x7fu; /* only reachable without saturation */
  return (uint8_t)(sign | bits);
}

/* __hip_fp8_e4m3(float) / __hip_fp8_e5m2(float) with __HIP_SATFINITE */
static uint8_t fp8_encode_sat(float f, int e5m2) {
  uint32_t x = f2u(f);
  if ((x & 0x7f800000u) != 0x7f800000u) {
    float m = e5m2 ? 57344.0f : 448.0f;
    if (f > m) f = m;
    if (f < -m) f = -m;
  }
  return fp8_encode_hw(f, e5m2);
}

/* software fp8 -> half of amd_hip_fp8.h:403-541: exact, every NaN -> +0x7C01, e5m2 inf -> inf */
static uint16_t fp8_to_half_sw(uint8_t b, int e5m2) {
  if (!e5m2 && (b & 0x7fu) == 0x7fu) return 0x7c01u;
  if (e5m2 && (b & 0x7cu) == 0x7cu && (b & 3u)) return 0x7c01u;
  if (e5m2) return (uint16_t)((uint16_t)b << 8);
  return float_to_half_rne(fp8_decode(b, 0));
}

/* __half add / compare without clip (calElements<__half>, reduce_kernel.hpp:16-24) */
static uint16_t half_add_noclip(uint16_t a, uint16_t b) {
  if (half_isnan(a) || half_isnan(b)) return 0x7e00u; /* a quiet +NaN: only its NaN-ness reaches fp8 */
  return float_to_half_rne(half_to_float(a) + half_to_float(b));
}
static uint16_t half_lt_min(uint16_t a, uint16_t b) { return half_to_float(a) < half_to_float(b) ? a : b; }

uint8_t oracle_fp8_encode_sat(float f, int e5m2) { return fp8_encode_sat(f, e5m2); }
float oracle_fp8_decode(uint8_t b, int e5m2) { return fp8_decode(b, e5m2); }

/* device fminf (v_min_f32, IEEE mode): a NaN operand yields the other one, and -0 < +0 */
static float fminf_dev(float x, float y) {
  if (x == y) return u2f(f2u(x) | f2u(y));
  return fminf(x, y);
}

/* T == AccumT (gpu_data_types.hpp:425-443, 499-516 with clip :353-371, min :690-750) */
static uint8_t fp8_reduce_same(uint8_t a, uint8_t b, int e5m2, int op) {
  float x = fp8_decode(a, e5m2), y = fp8_decode(b, e5m2);
  if (op == ORC_MIN) return fp8_encode_sat(fminf_dev(x, y), e5m2);
  uint8_t s = fp8_encode_sat(x + y, e5m2);
  if (!e5m2) return s; /* clip<__fp8_e4m3> is the identity */
  float f = fmaxf(fp8_decode(s, 1), -57344.0f); /* NaN -> -57344 */
  f = fminf(f, 57344.0f);
  return fp8_encode_sat(f, 1);
}

/* ---- e4m3b15 (gpu_data_types.hpp:78-155): software fp8, bias 15, no inf / NaN ----------------
 * decode (toFloat, :111-125): the fp16 bits sign | (byte & 0x7f) << 7, exact.
 * encode (fromFloat, :131-154): RNE to fp16, |h| clamped to 0x3f80 (1.875), then the upper byte of
 * (|h| * 2 + 0x80) with h's sign: the three kept mantissa bits rounded half up.  The gfx950 build
 * takes the generic branches of the vector conversions (:1016-1265), which reduce to these two. */
static uint16_t b15_to_h16(uint8_t b) { return (uint16_t)(((b & 0x80u) << 8) | ((b & 0x7fu) << 7)); }
static float b15_decode(uint8_t b) { return half_to_float(b15_to_h16(b)); }
static uint8_t b15_from_h16(uint16_t h) {
  uint32_t a = h & 0x7fffu;
  if (a > 0x3f80u) a = 0x3f80u;
  return (uint8_t)((((a * 2u + 0x80u) | (h & 0x8000u)) >> 8) & 0xffu);
}
static uint8_t b15_encode(float f) { return b15_from_h16(float_to_half_rne(f)); }
uint8_t oracle_b15_encode(float f) { return b15_encode(f); }
float oracle_b15_decode(uint8_t b) { return b15_decode(b); }

/* T == AccumT (:1269-1300): a + b = enc(dec(a) + dec(b)); min = enc(fminf(dec(a), dec(b))) */
static uint8_t b15_reduce_same(uint8_t a, uint8_t b, int op) {
  float x = b15_decode(a), y = b15_decode(b);
  return b15_encode(op == ORC_MIN ? fminf_dev(x, y) : x + y);
}

/* uint8 (gpu_data_types.hpp:577-589, :622-640): wrapping add, unsigned min */
static uint8_t u8_reduce(uint8_t a, uint8_t b, int op) {
  if (op == ORC_SUM) return (uint8_t)(a + b);
  return a < b ? a : b;
}

static void b15_reduce_seq(int dt, int op, int nsrc, const uint8_t* const* src, size_t nbytes, uint8_t* dst) {
  int kind = orc_acc_kind(dt);
  for (size_t i = 0; i < nbytes; i++) {
    if (kind == 0) {
      uint8_t a = src[0][i];
      for (int k = 1; k < nsrc; k++) a = b15_reduce_same(a, src[k][i], op);
      dst[i] = a;
    } else if (kind == 2) { /* AccumT float: up = dec, float add / (a < v ? a : v), down = enc */
      float a = b15_decode(src[0][i]);
      for (int k = 1; k < nsrc; k++) {
        float v = b15_decode(src[k][i]);
        a = (op == ORC_SUM) ? a + v : (a < v ? a : v);
      }
      dst[i] = b15_encode(a);
    } else { /* AccumT half: up = the exact fp16 image, __half add / compare, down = enc(half) */
      uint16_t a = b15_to_h16(src[0][i]);
      for (int k = 1; k < nsrc; k++) {
        uint16_t v = b15_to_h16(src[k][i]);
        a = (op == ORC_SUM) ? half_add_noclip(a, v) : half_lt_min(a, v);
      }
      dst[i] = b15_from_h16(a);
    }
  }
}

/* dst[i] = down(up(src[0][i]) (op) up(src[1][i]) (op) ...) for the 1-byte reduce types (OCP fp8,
 * e4m3b15, uint8), nsrc sources in sum order, over nbytes elements (calVectorAccum,
 * reduce_kernel.hpp:171-189). */
static void fp8_reduce_seq(int dt, int op, int nsrc, const uint8_t* const* src, size_t nbytes, uint8_t* dst) {
  if (orc_is_b15(dt)) {
    b15_reduce_seq(dt, op, nsrc, src, nbytes, dst);
    return;
  }
  if (dt == ORC_U8) {
    for (size_t i = 0; i < nbytes; i++) {
      uint8_t a = src[0][i];
      for (int k = 1; k < nsrc; k++) a = u8_reduce(a, src[k][i], op);
      dst[i] = a;
    }
    return;
  }
  int e5 = orc_is_e5m2(dt), kind = orc_acc_kind(dt);
  for (size_t i = 0; i < nbytes; i++) {
    if (kind == 0) {
      uint8_t a = src[0][i];
      for (int k = 1; k < nsrc; k++) a = fp8_reduce_same(a, src[k][i], e5, op);
      dst[i] = a;
    } else if (kind == 2) {
      float a = fp8_decode(src[0][i], e5);
      for (int k = 1; k < nsrc; k++) {
        float v = fp8_decode(src[k][i], e5);
        a = (op == ORC_SUM) ? a + v : (a < v ? a : v);
      }
      dst[i] = fp8_encode_sat(a, e5);
    } else {
      uint16_t a = fp8_to_half_sw(src[0][i], e5);
      for (int k = 1; k < nsrc; k++) {
        uint16_t v = fp8_to_half_sw(src[k][i], e5);
        a = (op == ORC_SUM) ? half_add_noclip(a, v) : half_lt_min(a, v);
      }
      dst[i] = fp8_encode_sat(half_to_float(a), e5);
    }
  }
}

/* calVectorAccum<T,T,Op> over one 32-bit word (reduce_kernel.hpp:86-134, 171-175). */
static uint32_t reduce_word(int dtype, int op, uint32_t acc, uint32_t val) {
  if (orc_is_byte(dtype)) { /* one accumulation step: down(up(acc) (op) up(val)) per byte */
    uint8_t a[4], v[4], r[4];
    const uint8_t* s[2] = {a, v};
    memcpy(a, &acc, 4);
    memcpy(v, &val, 4);
    fp8_reduce_seq(dtype, op, 2, s, 4, r);
    uint32_t out;
    memcpy(&out, r, 4);
    return out;
  }
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

/* dst = src[0] (op) src[1] (op) ... (op) src[nsrc-1], in this order, accumulating in the reduce
 * type's AccumT (upcastVector / calVectorAccum / downcastVector, reduce_kernel.hpp:139-189).
 * dst may alias src[0]. */
void oracle_reduce_seq(int dtype, int op, int nsrc, const uint32_t* const* src, size_t nwords, uint32_t* dst) {
  if (orc_is_byte(dtype)) {
    fp8_reduce_seq(dtype, op, nsrc, (const uint8_t* const*)src, nwords * 4, (uint8_t*)dst);
    return;
  }
  if (dst != src[0]) memmove(dst, src[0], nwords * 4);
  for (int k = 1; k < nsrc; k++) oracle_reduce_words(dtype, op, dst, src[k], nwords);
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
  uint64_t W = orc_ll_words(dtype, count); /* :51-54 */
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
  uint32_t* tmp = (uint32_t*)malloc((size_t)n * (wpr * 4 + 8));
  for (int r = 0; r < n; r++) {
    uint32_t* acc = out[r] + (uint64_t)r * wpr;
    const uint32_t* srcs[64];
    int ns = 0;
    srcs[ns++] = in[r] + (uint64_t)r * wpr; /* own copy first, then peers ascending */
    for (int p = 0; p < n; p++) {
      if (p == r) continue;
      const uint32_t* pk = scratch[r] + (base + (uint64_t)p * ppr * 16) / 4;
      uint32_t* t = tmp + (size_t)ns * (wpr + 2);
      oracle_ll16_unpack(pk, ppr, flag, t);
      srcs[ns++] = t;
    }
    oracle_reduce_seq(dtype, op, ns, srcs, wpr, acc);
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

/* mscclpp-test allreduce6 / allreduce7 (test/mscclpp-test/allreduce_test.cu:972-1093), int32.
 * nelemsPerRank = nelems / n (the host requires it even); 16-byte packets in the harness layout:
 * input region at packet (flag & 1 ? 0 : nPkts), result region at packet (flag & 1 ? 2 : 3) * nPkts
 * (:987-991; k7's 8-byte LL8 packets at (flag & 1 ? 0 : nelems) etc. are the same bytes, :1048-1051).
 * Sum: 0 + peers ascending + own (:999-1010), wrapping int32 adds. */
void oracle_mscclpp_test_ll(int n, const uint32_t* const* in, uint64_t nelems, uint32_t flag,
                            uint32_t* const* scratch, uint32_t* const* out) {
  uint64_t nPkts = nelems / 2, epr = nelems / (uint64_t)n, ppr = epr / 2;
  uint64_t inBase = (flag & 1u) ? 0 : nPkts, resBase = (flag & 1u) ? 2 * nPkts : 3 * nPkts;
  for (int s = 0; s < n; s++) /* step 1 */
    for (int q = 0; q < n; q++)
      if (q != s) oracle_ll16_pack(in[s] + (uint64_t)q * epr, ppr, flag, scratch[q] + (inBase + (uint64_t)s * ppr) * 4);
  uint32_t* tmp = (uint32_t*)malloc(epr * 4 + 8);
  uint32_t* acc = (uint32_t*)malloc(epr * 4 + 8);
  for (int r = 0; r < n; r++) { /* step 2 */
    memset(acc, 0, epr * 4);
    for (int p = 0; p < n; p++) {
      if (p == r) continue;
      oracle_ll16_unpack(scratch[r] + (inBase + (uint64_t)p * ppr) * 4, ppr, flag, tmp);
      for (uint64_t i = 0; i < epr; i++) acc[i] += tmp[i];
    }
    for (uint64_t i = 0; i < epr; i++) acc[i] += in[r][(uint64_t)r * epr + i];
    memcpy(out[r] + (uint64_t)r * epr, acc, epr * 4);
    for (int q = 0; q < n; q++)
      if (q != r) oracle_ll16_pack(acc, ppr, flag, scratch[q] + (resBase + (uint64_t)r * ppr) * 4);
  }
  for (int r = 0; r < n; r++) /* step 3 */
    for (int p = 0; p < n; p++)
      if (p != r) oracle_ll16_unpack(scratch[r] + (resBase + (uint64_t)p * ppr) * 4, ppr, flag, out[r] + (uint64_t)p * epr);
  free(tmp);
  free(acc);
}

/* One 32-bit word of python/mscclpp_benchmark/allreduce.cu's add_vectors<TYPE>(a, b) (:37-96):
 * TYPE=int wrapping add, TYPE=float `a + b` (RNE, no clip), TYPE=__half __hadd2 on the word's two
 * halves (RNE, no clip: inf on overflow, a NaN operand propagates, quieted, with its payload). */
static uint32_t bench_add_word(int dtype, uint32_t a, uint32_t b) {
  if (dtype == ORC_F32) return f2u(u2f(a) + u2f(b));
  if (dtype == ORC_F16) {
    uint16_t lo = float_to_half_rne(half_to_float((uint16_t)a) + half_to_float((uint16_t)b));
    uint16_t hi = float_to_half_rne(half_to_float((uint16_t)(a >> 16)) + half_to_float((uint16_t)(b >> 16)));
    return (uint32_t)lo | ((uint32_t)hi << 16);
  }
  return a + b;
}

/* python/mscclpp_benchmark/allreduce.cu:223-289 allreduce2 for TYPE = int (ORC_I32), float (ORC_F32)
 * or __half (ORC_F16), on one node; nwords = the rank's buffer in 32-bit words (the kernel's nelems
 * after its `nelems / (sizeof(int) / sizeof(TYPE))`, :229).  Same packets and scratch layout as
 * allreduce6 above (:239-248); per 32-bit word the reduction is, as the kernel orders its operands,
 *   order 0:  data = 0;  data = val_p + data  for peers p ascending (:257-262);  data = data + own (:263)
 * and, only to show that the test can tell orders apart,
 *   order 1:  data = own;  data = data + val_p  for peers p ascending.
 * A float/half 0 + (-0) is +0, so order 0 turns an all-(-0) word into +0 where order 1 keeps -0. */
void oracle_bench_allreduce2(int dtype, int order, int n, const uint32_t* const* in, uint64_t nwords, uint32_t flag,
                             uint32_t* const* scratch, uint32_t* const* out) {
  uint64_t nPkts = nwords / 2, epr = nwords / (uint64_t)n, ppr = epr / 2;
  uint64_t inBase = (flag & 1u) ? 0 : nPkts, resBase = (flag & 1u) ? 2 * nPkts : 3 * nPkts;
  for (int s = 0; s < n; s++) /* step 1 */
    for (int q = 0; q < n; q++)
      if (q != s) oracle_ll16_pack(in[s] + (uint64_t)q * epr, ppr, flag, scratch[q] + (inBase + (uint64_t)s * ppr) * 4);
  uint32_t* tmp = (uint32_t*)malloc(epr * 4 + 8);
  uint32_t* acc = (uint32_t*)malloc(epr * 4 + 8);
  for (int r = 0; r < n; r++) { /* step 2 */
    const uint32_t* own = in[r] + (uint64_t)r * epr;
    if (order == 0) memset(acc, 0, epr * 4);
    else memcpy(acc, own, epr * 4);
    for (int p = 0; p < n; p++) {
      if (p == r) continue;
      oracle_ll16_unpack(scratch[r] + (inBase + (uint64_t)p * ppr) * 4, ppr, flag, tmp);
      for (uint64_t i = 0; i < epr; i++)
        acc[i] = order == 0 ? bench_add_word(dtype, tmp[i], acc[i]) : bench_add_word(dtype, acc[i], tmp[i]);
    }
    if (order == 0)
      for (uint64_t i = 0; i < epr; i++) acc[i] = bench_add_word(dtype, acc[i], own[i]);
    memcpy(out[r] + (uint64_t)r * epr, acc, epr * 4);
    for (int q = 0; q < n; q++)
      if (q != r) oracle_ll16_pack(acc, ppr, flag, scratch[q] + (resBase + (uint64_t)r * ppr) * 4);
  }
  for (int r = 0; r < n; r++) /* step 3 */
    for (int p = 0; p < n; p++)
      if (p != r) oracle_ll16_unpack(scratch[r] + (resBase + (uint64_t)p * ppr) * 4, ppr, flag, out[r] + (uint64_t)p * epr);
  free(tmp);
  free(acc);
}

/* python/mscclpp_benchmark/allreduce.cu:123-221 allreduce1 (TYPE = int, float or __half), in place,
 * for a chunk of nwords / n words per rank that is a whole number of int4 vectors (the kernel's
 * remainder path is then empty, :166-185).  The owner r of chunk r reduces it as the kernel orders
 * its operands (:147-156): tmp = own; for index = 0 .. n - 2: p = (index + r) mod (n - 1), the
 * channel to rank p < r ? p : p + 1, tmp = tmp + that rank's chunk; every rank's buffer ends holding
 * tmp in chunk r (written to the peers, :158-164, and to the own buffer, :165). */
void oracle_bench_allreduce1(int dtype, int n, const uint32_t* const* in, uint64_t nwords, uint32_t* const* out) {
  const uint64_t cw = nwords / (uint64_t)n;
  const int nPeer = n - 1;
  for (int r = 0; r < n; r++) {
    for (uint64_t i = r * cw; i < (uint64_t)(r + 1) * cw; i++) {
      uint32_t tmp = in[r][i];
      for (int index = 0; index < nPeer; index++) {
        int peerIdx = index + r;
        if (peerIdx >= nPeer) peerIdx -= nPeer;
        const int remote = peerIdx < r ? peerIdx : peerIdx + 1;
        tmp = bench_add_word(dtype, tmp, in[remote][i]);
      }
      for (int q = 0; q < n; q++) out[q][i] = tmp;
    }
  }
}

/* mscclpp-test allreduce2, single node (test/mscclpp-test/allreduce_test.cu:841-943, worldSize ==
 * nRanksPerNode), int32, nelems even.  One hop of LL16 packets (LLPacket = {x, flag, y, flag}):
 * rank s puts its whole buffer into every peer q's scratch at packet
 * scratchBaseIndex + (s < q ? s : s - 1) * nPkts, scratchBaseIndex = flag & 1 ? 0 : nPkts * (n - 1)
 * (:861-863, :876-880); rank r sums the n - 1 packet streams in slot order from 0 and adds its own
 * input last (:884-904), wrapping int32 adds; the result goes to the separate result buffer. */
void oracle_mscclpp_test_k2(int n, const uint32_t* const* in, uint64_t nelems, uint32_t flag,
                            uint32_t* const* scratch, uint32_t* const* out) {
  const uint64_t nPkts = nelems / 2, nPeers = (uint64_t)(n - 1);
  const uint64_t base = (flag & 1u) ? 0 : nPkts * nPeers;
  for (int s = 0; s < n; s++)
    for (int q = 0; q < n; q++)
      if (q != s) {
        const uint64_t slot = (uint64_t)(s < q ? s : s - 1);
        oracle_ll16_pack(in[s], nPkts, flag, scratch[q] + (base + slot * nPkts) * 4);
      }
  uint32_t* tmp = (uint32_t*)malloc(nelems * 4 + 8);
  for (int r = 0; r < n; r++) {
    for (uint64_t i = 0; i < nelems; i++) out[r][i] = 0;
    for (uint64_t slot = 0; slot < nPeers; slot++) {
      oracle_ll16_unpack(scratch[r] + (base + slot * nPkts) * 4, nPkts, flag, tmp);
      for (uint64_t i = 0; i < nelems; i++) out[r][i] += tmp[i];
    }
    for (uint64_t i = 0; i < nelems; i++) out[r][i] = in[r][i] + out[r][i];
  }
  free(tmp);
}

/* allreduceAllPairs (allreduce_allpair_packet.cu:15-69): one-hop LL8.  Rank s writes its
 * whole buffer (W words, W=(2c+2)/4 for 2-byte types) as LL8 packets into every peer's scratch
 * at s*W packets (:28, :40-41); rank r sums x_r then peers ascending (:49-61). */
void oracle_allreduce_allpairs(int dtype, int op, int n, const uint32_t* const* in, uint64_t count,
                               uint32_t flag, uint64_t half_bytes, uint32_t* const* scratch,
                               uint32_t* const* out) {
  uint64_t W = orc_ll_words(dtype, count);
  uint64_t base = (flag % 2) ? half_bytes : 0;
  for (int s = 0; s < n; s++)
    for (int q = 0; q < n; q++) {
      if (q == s) continue;
      oracle_ll8_pack(in[s], W, flag, scratch[q] + (base + (uint64_t)s * W * 8) / 4);
    }
  uint32_t* tmp = (uint32_t*)malloc((size_t)n * (W * 4 + 8));
  for (int r = 0; r < n; r++) {
    const uint32_t* srcs[64];
    int ns = 0;
    srcs[ns++] = in[r]; /* own first, then peers ascending (:51-60) */
    for (int p = 0; p < n; p++) {
      if (p == r) continue;
      uint32_t* t = tmp + (size_t)ns * (W + 2);
      oracle_ll8_unpack(scratch[r] + (base + (uint64_t)p * W * 8) / 4, W, flag, t);
      srcs[ns++] = t;
    }
    oracle_reduce_seq(dtype, op, ns, srcs, W, out[r]);
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
  const uint32_t* srcs[64];
  int ns = 0;
  srcs[ns++] = in[start] + w0;
  if (order_kind == 0) {
    for (int p = 0; p < n; p++)
      if (p != owner) srcs[ns++] = in[p] + w0;
  } else {
    for (int k = 1; k < n; k++) srcs[ns++] = in[(start + k) % n] + w0;
  }
  oracle_reduce_seq(dtype, op, ns, srcs, nw, dst);
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

/* The AllReduce result (one output buffer) when word w belongs to owner (w mod period) / chunk and
 * is reduced by that owner in `order_kind` order:
 *   period = n * slice, chunk = slice            contiguous slices (fullmesh kind 0, rsag kind 1)
 *   period = n * 4C,    chunk = 4C words         allreduceRsAgPipeline's interleaved slots
 *                                                (allreduce_rsag_pipeline.cu:104-117, C units of 16 B)
 * With period >= nwords and slice = ceil-to-16-bytes this equals oracle_allreduce_sliced. */
void oracle_allreduce_owned(int dtype, int op, int n, const uint32_t* const* in, uint64_t nwords,
                            uint64_t period_words, uint64_t chunk_words, int order_kind, uint32_t* out) {
  for (uint64_t w0 = 0; w0 < nwords; w0 += chunk_words) {
    const int owner = (int)((w0 % period_words) / chunk_words);
    uint64_t nw = chunk_words;
    if (w0 + nw > nwords) nw = nwords - w0;
    reduce_range(dtype, op, n, in, owner < n ? owner : n - 1, order_kind, w0, nw, out + w0);
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
    else if (orc_is_fp8(dtype))
      ((uint8_t*)dst)[i] = fp8_encode_sat(v, orc_is_e5m2(dtype));
    else if (orc_is_b15(dtype))
      ((uint8_t*)dst)[i] = b15_encode(v);
    else if (dtype == ORC_U8)
      ((uint8_t*)dst)[i] = (uint8_t)(s % 4096 >> 4);
    else
      ((uint32_t*)dst)[i] = (uint32_t)(int32_t)(v * 2147483647.0f);
  }
}
