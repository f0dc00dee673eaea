// Element-wise reduction over packed 32-bit words, bit-compatible with the reference's
// calVectorAccum<T, T, Op> (src/core/include/reduce_kernel.hpp:16-189) and the operators in
// include/mscclpp/gpu_data_types.hpp:315-420, 588-620:
//   fp16 SUM : clip(__hadd2(a, b))  -> v_pk_add_f16, then v_pk_max_f16 / v_pk_min_f16 against
//              +-65504 (maxNum/minNum return the non-NaN operand, so NaN -> -65504, +-inf -> +-65504)
//   bf16 SUM : clip(__hadd2(a, b))  -> f32 add + v_cvt_pk_bf16_f32 (RNE), bounds +-inf: NaN -> -inf
//   fp32 SUM : plain RNE add (v_pk_add_f32 on pairs), no clip
//   int32/uint32 SUM : wrapping add
//   MIN : __hmin / fminf semantics, including the tie and NaN rules of
//         /opt/rocm/include/hip/amd_detail/amd_hip_fp16.h:768-775 and amd_hip_bf16.h:1308-1315
// No MFMA: the sum is a vertical element-wise add, not a contraction.
#pragma once

#include "device.hpp"

namespace mscclpp_amd {

// Reduce types.  0..4 and 11 accumulate in the element type.  The FP8 codes (OCP e4m3 / e5m2, the
// gfx950 hardware formats, and the software e4m3b15) carry the accumulation type of
// calVectorAccum<T, AccumT, Op> (reduce_kernel.hpp:171-189, dispatchFp8Accum common.hpp:89-100):
// T, half or float.  The dispatch of dispatchByDtype (common.hpp:103-135) on gfx950 is complete with
// these: fp16, fp32, bf16, OCP e4m3 / e5m2, e4m3b15, int32 / uint32, uint8.
enum DType : int {
  kF16 = 0, kBF16 = 1, kF32 = 2, kI32 = 3, kU32 = 4,
  kE4M3 = 5, kE5M2 = 6,              // AccumT = T
  kE4M3AccF16 = 7, kE5M2AccF16 = 8,  // AccumT = half
  kE4M3AccF32 = 9, kE5M2AccF32 = 10, // AccumT = float
  kU8 = 11,                          // uint8_t (Adapter<Op, uint8_t, uint8_t>, common.hpp:132-133)
  kB15 = 12, kB15AccF16 = 13, kB15AccF32 = 14  // __fp8_e4m3b15, AccumT = T / half / float
};
enum ROp : int { kSum = 0, kMin = 1 };

__host__ __device__ constexpr bool is_fp8(int dt) { return dt >= kE4M3 && dt <= kE5M2AccF32; }  // OCP, hardware
__host__ __device__ constexpr bool is_b15(int dt) { return dt >= kB15 && dt <= kB15AccF32; }
__host__ __device__ constexpr bool is_e5m2(int dt) { return dt == kE5M2 || dt == kE5M2AccF16 || dt == kE5M2AccF32; }
__host__ __device__ constexpr int elem_bytes(int dt) {
  return (dt == kF16 || dt == kBF16) ? 2 : ((is_fp8(dt) || is_b15(dt) || dt == kU8) ? 1 : 4);
}

typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
typedef float float2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ half2_t as_h2(uint32_t w) { return __builtin_bit_cast(half2_t, w); }
__device__ __forceinline__ uint32_t from_h2(half2_t h) { return __builtin_bit_cast(uint32_t, h); }

__device__ __forceinline__ uint32_t f16x2_add_clip(uint32_t a, uint32_t b) {
  half2_t s = as_h2(a) + as_h2(b);
  const half2_t lo = {(_Float16)-65504.0f, (_Float16)-65504.0f};
  const half2_t hi = {(_Float16)65504.0f, (_Float16)65504.0f};
  s = __builtin_elementwise_min(__builtin_elementwise_max(s, lo), hi);
  return from_h2(s);
}

__device__ __forceinline__ float bf16_lo(uint32_t w) { return __builtin_bit_cast(float, w << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t w) { return __builtin_bit_cast(float, w & 0xffff0000u); }

__device__ __forceinline__ uint32_t bf16x2_add_clip(uint32_t a, uint32_t b) {
  __bf16 r0 = (__bf16)(bf16_lo(a) + bf16_lo(b));
  __bf16 r1 = (__bf16)(bf16_hi(a) + bf16_hi(b));
  uint32_t u0 = __builtin_bit_cast(uint16_t, r0), u1 = __builtin_bit_cast(uint16_t, r1);
  // clip<__bfloat16>: only NaN changes (to -inf): __hmax(NaN, -inf) = -inf, __hmin(-inf, inf) = -inf.
  if ((u0 & 0x7fffu) > 0x7f80u) u0 = 0xff80u;
  if ((u1 & 0x7fffu) > 0x7f80u) u1 = 0xff80u;
  return u0 | (u1 << 16);
}

__device__ __forceinline__ uint32_t h16_min(uint32_t x, uint32_t y) {
  // __hmin: NaN yields the other operand, both NaN -> 0x7fff, x > y ? y : x.
  bool nx = (x & 0x7fffu) > 0x7c00u, ny = (y & 0x7fffu) > 0x7c00u;
  if (nx && ny) return 0x7fffu;
  if (nx) return y;
  if (ny) return x;
  _Float16 fx = __builtin_bit_cast(_Float16, (uint16_t)x), fy = __builtin_bit_cast(_Float16, (uint16_t)y);
  return fx > fy ? y : x;
}
__device__ __forceinline__ uint32_t bf16_min1(uint32_t a, uint32_t b) {
  // bf16 __hmin: NaN yields the other operand, both NaN -> 0x7fff, a < b ? a : b.
  bool na = (a & 0x7fffu) > 0x7f80u, nb = (b & 0x7fffu) > 0x7f80u;
  if (na && nb) return 0x7fffu;
  if (na) return b;
  if (nb) return a;
  float fa = __builtin_bit_cast(float, a << 16), fb = __builtin_bit_cast(float, b << 16);
  return fa < fb ? a : b;
}

// ---- OCP FP8 on gfx950 ---------------------------------------------------------------------
// The reference's gfx950 build takes the generic branches of gpu_data_types.hpp (its packed fp8
// paths are gfx942-only), i.e. per element:
//   decode  float(fp8)          -> v_cvt_f32_fp8 / v_cvt_f32_bf8  (amd_hip_fp8.h:638-650)
//   encode  __hip_fp8_*(float)  -> saturate non-NaN/Inf to +-448 / +-57344 with v_med3_f32, then
//                                  v_cvt_pk_fp8_f32 / v_cvt_pk_bf8_f32, RNE (amd_hip_fp8.h:548-592)
//   T == AccumT:  e4m3 a+b = enc(dec(a)+dec(b))                        (gpu_data_types.hpp:425-443)
//                 e5m2 a+b = clip(enc(dec(a)+dec(b))), clip = enc(fminf(fmaxf(dec, -57344), 57344))
//                                                                      (:499-516, :362-371)
//                 min(a,b) = enc(fminf(dec(a), dec(b)))                 (:690-750)
//   AccumT float: up = dec, acc+v / (acc < v ? acc : v), down = enc      (reduce_kernel.hpp:139-189,
//                                                                        gpu_data_types.hpp:758-948)
//   AccumT half:  up = software fp8->half (NaN -> +0x7C01, amd_hip_fp8.h:403-541), __half add /
//                 (a < b ? a : b), down = enc(float(h))                  (gpu_data_types.hpp:957-1004)
typedef _Float16 half4_t __attribute__((ext_vector_type(4)));
typedef float float4_t __attribute__((ext_vector_type(4)));

template <bool E5M2>
__device__ __forceinline__ float4_t fp8x4_decode(uint32_t w) {
  float2_t lo, hi;
  if constexpr (E5M2) {
    lo = __builtin_amdgcn_cvt_pk_f32_bf8((int)w, false);
    hi = __builtin_amdgcn_cvt_pk_f32_bf8((int)w, true);
  } else {
    lo = __builtin_amdgcn_cvt_pk_f32_fp8((int)w, false);
    hi = __builtin_amdgcn_cvt_pk_f32_fp8((int)w, true);
  }
  return float4_t{lo.x, lo.y, hi.x, hi.y};
}

template <bool E5M2>
__device__ __forceinline__ float fp8_sat(float v) {
  constexpr float m = E5M2 ? 57344.0f : 448.0f;
  if ((__builtin_bit_cast(uint32_t, v) & 0x7f800000u) != 0x7f800000u) v = __builtin_amdgcn_fmed3f(v, m, -m);
  return v;
}

template <bool E5M2>
__device__ __forceinline__ uint32_t fp8x4_encode(float4_t f) {
  const float a = fp8_sat<E5M2>(f.x), b = fp8_sat<E5M2>(f.y), c = fp8_sat<E5M2>(f.z), d = fp8_sat<E5M2>(f.w);
  if constexpr (E5M2) {
    int r = __builtin_amdgcn_cvt_pk_bf8_f32(a, b, 0, false);
    return (uint32_t)__builtin_amdgcn_cvt_pk_bf8_f32(c, d, r, true);
  } else {
    int r = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
    return (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(c, d, r, true);
  }
}

// software fp8 -> half of amd_hip_fp8.h:403-541 (exact; every NaN becomes +0x7C01)
template <bool E5M2>
__device__ __forceinline__ _Float16 fp8_to_half_sw(uint32_t b, float hw) {
  const bool nan = E5M2 ? ((b & 0x7cu) == 0x7cu && (b & 3u)) : ((b & 0x7fu) == 0x7fu);
  return nan ? __builtin_bit_cast(_Float16, (uint16_t)0x7c01u) : (_Float16)hw;
}
template <bool E5M2>
__device__ __forceinline__ half4_t fp8x4_to_half4(uint32_t w) {
  const float4_t f = fp8x4_decode<E5M2>(w);
  return half4_t{fp8_to_half_sw<E5M2>(w & 0xffu, f.x), fp8_to_half_sw<E5M2>((w >> 8) & 0xffu, f.y),
                 fp8_to_half_sw<E5M2>((w >> 16) & 0xffu, f.z), fp8_to_half_sw<E5M2>(w >> 24, f.w)};
}

template <int OP>
__device__ __forceinline__ float4_t acc_op(float4_t a, float4_t b) {
  if constexpr (OP == kSum) return a + b;
  return float4_t{a.x < b.x ? a.x : b.x, a.y < b.y ? a.y : b.y, a.z < b.z ? a.z : b.z, a.w < b.w ? a.w : b.w};
}
template <int OP>
__device__ __forceinline__ half4_t acc_op(half4_t a, half4_t b) {
  if constexpr (OP == kSum) return a + b;
  return half4_t{a.x < b.x ? a.x : b.x, a.y < b.y ? a.y : b.y, a.z < b.z ? a.z : b.z, a.w < b.w ? a.w : b.w};
}

// T == AccumT fp8 (4 elements per word)
template <bool E5M2, int OP>
__device__ __forceinline__ uint32_t fp8x4_reduce(uint32_t a, uint32_t b) {
  const float4_t x = fp8x4_decode<E5M2>(a), y = fp8x4_decode<E5M2>(b);
  if constexpr (OP == kMin) {
    return fp8x4_encode<E5M2>(float4_t{fminf(x.x, y.x), fminf(x.y, y.y), fminf(x.z, y.z), fminf(x.w, y.w)});
  } else {
    const uint32_t s = fp8x4_encode<E5M2>(x + y);
    if constexpr (!E5M2) return s;
    // clip<__fp8_e5m2>: NaN -> -57344 (fmaxf drops the NaN), +-inf -> +-57344
    const float4_t f = fp8x4_decode<E5M2>(s);
    const float4_t c = {fminf(fmaxf(f.x, -57344.0f), 57344.0f), fminf(fmaxf(f.y, -57344.0f), 57344.0f),
                        fminf(fmaxf(f.z, -57344.0f), 57344.0f), fminf(fmaxf(f.w, -57344.0f), 57344.0f)};
    return fp8x4_encode<E5M2>(c);
  }
}

// ---- uint8 (gpu_data_types.hpp:577-589, :622-640): four lanes per word, wrapping add and
// unsigned min per byte -------------------------------------------------------------------------
__device__ __forceinline__ uint32_t u8x4_add(uint32_t a, uint32_t b) {
  constexpr uint32_t even = 0x00ff00ffu;
  return (((a & even) + (b & even)) & even) | (((a & ~even) + (b & ~even)) & ~even);
}
__device__ __forceinline__ uint32_t u8x4_min(uint32_t a, uint32_t b) {
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    const uint32_t x = (a >> k) & 0xffu, y = (b >> k) & 0xffu;
    r |= (x < y ? x : y) << k;
  }
  return r;
}

// ---- e4m3b15: software fp8, bias 15, no inf / NaN (gpu_data_types.hpp:78-155, 1008-1300) --------
// decode: the fp16 bits sign | (byte & 0x7f) << 7 (exponent E4 -> E5, same bias), exact;
// encode from fp16 h: |h| clamped to 0x3f80 (1.875), then (|h| * 2 + 0x80) >> 8 with h's sign --
// a round-half-up of the three kept mantissa bits; from float: RNE to fp16 first (fromFloat).
// The gfx950 build takes the reference's generic branches (its packed paths are gfx942 / CUDA):
//   T == AccumT:  a + b = enc(dec(a) + dec(b)) in float; min = enc(fminf(dec(a), dec(b)))
//   AccumT half:  up = dec as fp16, plain __half add / (a < b ? a : b), down = enc(half)
//   AccumT float: up = dec, float add / (a < b ? a : b), down = enc(float)
__device__ __forceinline__ uint32_t b15_to_h16(uint32_t b) { return ((b & 0x80u) << 8) | ((b & 0x7fu) << 7); }
__device__ __forceinline__ uint32_t b15_from_h16(uint32_t h) {
  uint32_t a = h & 0x7fffu;
  a = a < 0x3f80u ? a : 0x3f80u;
  return (((a * 2u + 0x80u) | (h & 0x8000u)) >> 8) & 0xffu;
}
__device__ __forceinline__ half4_t b15x4_to_half4(uint32_t w) {
  return half4_t{__builtin_bit_cast(_Float16, (uint16_t)b15_to_h16(w & 0xffu)),
                 __builtin_bit_cast(_Float16, (uint16_t)b15_to_h16((w >> 8) & 0xffu)),
                 __builtin_bit_cast(_Float16, (uint16_t)b15_to_h16((w >> 16) & 0xffu)),
                 __builtin_bit_cast(_Float16, (uint16_t)b15_to_h16(w >> 24))};
}
__device__ __forceinline__ float4_t b15x4_decode(uint32_t w) {
  const half4_t h = b15x4_to_half4(w);
  return float4_t{(float)h.x, (float)h.y, (float)h.z, (float)h.w};
}
__device__ __forceinline__ uint32_t b15x4_from_half4(half4_t h) {
  // Bit-cast the whole vector: this clang (roc-7.2.0) lowers __builtin_bit_cast of an
  // ext_vector element lvalue (h.y, h.z, h.w) to a read of element 0.
  const u32x2 p = __builtin_bit_cast(u32x2, h);
  return b15_from_h16(p.x & 0xffffu) | (b15_from_h16(p.x >> 16) << 8) | (b15_from_h16(p.y & 0xffffu) << 16) |
         (b15_from_h16(p.y >> 16) << 24);
}
__device__ __forceinline__ uint32_t b15x4_encode(float4_t f) {  // float -> fp16 RNE -> e4m3b15
  return b15x4_from_half4(half4_t{(_Float16)f.x, (_Float16)f.y, (_Float16)f.z, (_Float16)f.w});
}
template <int OP>
__device__ __forceinline__ uint32_t b15x4_reduce(uint32_t a, uint32_t b) {
  const float4_t x = b15x4_decode(a), y = b15x4_decode(b);
  if constexpr (OP == kMin)
    return b15x4_encode(float4_t{fminf(x.x, y.x), fminf(x.y, y.y), fminf(x.z, y.z), fminf(x.w, y.w)});
  return b15x4_encode(x + y);
}

// Word accumulator: up(word) -> acc; add(acc, word) -> acc; down(acc) -> word.
template <int DT, int OP, int KIND = (DT == kE4M3AccF16 || DT == kE5M2AccF16) ? 1
                                     : (DT == kE4M3AccF32 || DT == kE5M2AccF32) ? 2
                                     : DT == kB15AccF16 ? 3
                                     : DT == kB15AccF32 ? 4 : 0>
struct AccWord;

template <int DT, int OP>
__device__ __forceinline__ uint32_t reduce_word(uint32_t acc, uint32_t val);

template <int DT, int OP>
struct AccWord<DT, OP, 0> {  // AccumT == T: the packed word itself
  static constexpr bool kWide = false;
  typedef uint32_t W;
  static __device__ __forceinline__ W up(uint32_t w) { return w; }
  static __device__ __forceinline__ W add(W a, uint32_t w) { return reduce_word<DT, OP>(a, w); }
  static __device__ __forceinline__ uint32_t down(W a) { return a; }
};
template <int DT, int OP>
struct AccWord<DT, OP, 1> {  // AccumT == half
  static constexpr bool kWide = true;
  typedef half4_t W;
  static __device__ __forceinline__ W up(uint32_t w) { return fp8x4_to_half4<is_e5m2(DT)>(w); }
  static __device__ __forceinline__ W add(W a, uint32_t w) { return acc_op<OP>(a, fp8x4_to_half4<is_e5m2(DT)>(w)); }
  static __device__ __forceinline__ uint32_t down(W a) {
    return fp8x4_encode<is_e5m2(DT)>(float4_t{(float)a.x, (float)a.y, (float)a.z, (float)a.w});
  }
};
template <int DT, int OP>
struct AccWord<DT, OP, 2> {  // AccumT == float
  static constexpr bool kWide = true;
  typedef float4_t W;
  static __device__ __forceinline__ W up(uint32_t w) { return fp8x4_decode<is_e5m2(DT)>(w); }
  static __device__ __forceinline__ W add(W a, uint32_t w) { return acc_op<OP>(a, fp8x4_decode<is_e5m2(DT)>(w)); }
  static __device__ __forceinline__ uint32_t down(W a) { return fp8x4_encode<is_e5m2(DT)>(a); }
};

template <int DT, int OP>
struct AccWord<DT, OP, 3> {  // e4m3b15, AccumT == half
  static constexpr bool kWide = true;
  typedef half4_t W;
  static __device__ __forceinline__ W up(uint32_t w) { return b15x4_to_half4(w); }
  static __device__ __forceinline__ W add(W a, uint32_t w) { return acc_op<OP>(a, b15x4_to_half4(w)); }
  static __device__ __forceinline__ uint32_t down(W a) { return b15x4_from_half4(a); }
};
template <int DT, int OP>
struct AccWord<DT, OP, 4> {  // e4m3b15, AccumT == float
  static constexpr bool kWide = true;
  typedef float4_t W;
  static __device__ __forceinline__ W up(uint32_t w) { return b15x4_decode(w); }
  static __device__ __forceinline__ W add(W a, uint32_t w) { return acc_op<OP>(a, b15x4_decode(w)); }
  static __device__ __forceinline__ uint32_t down(W a) { return b15x4_encode(a); }
};

// N-word accumulator over a u32x2 / u32x4 payload (the order of add() calls is the sum order).
template <int DT, int OP, int N>
struct Accum {
  typedef AccWord<DT, OP> A;
  typename A::W w[N];
  template <typename V>
  __device__ __forceinline__ explicit Accum(V v) {
#pragma unroll
    for (int i = 0; i < N; ++i) w[i] = A::up(v[i]);
  }
  template <typename V>
  __device__ __forceinline__ void add(V v) {
#pragma unroll
    for (int i = 0; i < N; ++i) w[i] = A::add(w[i], v[i]);
  }
  template <typename V>
  __device__ __forceinline__ V get() const {
    V r;
#pragma unroll
    for (int i = 0; i < N; ++i) r[i] = A::down(w[i]);
    return r;
  }
};

template <int DT, int OP>
__device__ __forceinline__ uint32_t reduce_word(uint32_t acc, uint32_t val) {
  if constexpr (DT == kE4M3 || DT == kE5M2) {
    return fp8x4_reduce<DT == kE5M2, OP>(acc, val);
  } else if constexpr (DT == kB15) {
    return b15x4_reduce<OP>(acc, val);
  } else if constexpr (DT == kU8) {
    return OP == kSum ? u8x4_add(acc, val) : u8x4_min(acc, val);
  } else if constexpr (is_fp8(DT) || is_b15(DT)) {
    // one accumulation step of calVectorAccum<T, AccumT>: down(up(acc) (op) up(val))
    typedef AccWord<DT, OP> A;
    return A::down(A::add(A::up(acc), val));
  } else if constexpr (OP == kSum) {
    if constexpr (DT == kF16) return f16x2_add_clip(acc, val);
    if constexpr (DT == kBF16) return bf16x2_add_clip(acc, val);
    if constexpr (DT == kF32) return __builtin_bit_cast(uint32_t, __builtin_bit_cast(float, acc) + __builtin_bit_cast(float, val));
    if constexpr (DT == kI32 || DT == kU32) return acc + val;
  } else {
    if constexpr (DT == kF16) return h16_min(acc & 0xffffu, val & 0xffffu) | (h16_min(acc >> 16, val >> 16) << 16);
    if constexpr (DT == kBF16) return bf16_min1(acc & 0xffffu, val & 0xffffu) | (bf16_min1(acc >> 16, val >> 16) << 16);
    if constexpr (DT == kF32)
      return __builtin_bit_cast(uint32_t, fminf(__builtin_bit_cast(float, acc), __builtin_bit_cast(float, val)));
    if constexpr (DT == kI32) return (int32_t)acc < (int32_t)val ? acc : val;
    if constexpr (DT == kU32) return acc < val ? acc : val;
  }
  return 0;
}

template <int DT, int OP>
__device__ __forceinline__ u32x4 reduce4(u32x4 a, u32x4 b) {
  if constexpr (DT == kF32 && OP == kSum) {
    // two v_pk_add_f32: the same RNE adds as four scalar adds
    float2_t lo = __builtin_bit_cast(float2_t, u32x2{a.x, a.y}) + __builtin_bit_cast(float2_t, u32x2{b.x, b.y});
    float2_t hi = __builtin_bit_cast(float2_t, u32x2{a.z, a.w}) + __builtin_bit_cast(float2_t, u32x2{b.z, b.w});
    u32x2 l = __builtin_bit_cast(u32x2, lo), h = __builtin_bit_cast(u32x2, hi);
    return u32x4{l.x, l.y, h.x, h.y};
  } else {
    u32x4 r;
    r.x = reduce_word<DT, OP>(a.x, b.x);
    r.y = reduce_word<DT, OP>(a.y, b.y);
    r.z = reduce_word<DT, OP>(a.z, b.z);
    r.w = reduce_word<DT, OP>(a.w, b.w);
    return r;
  }
}

// Runtime (dtype, op) -> template dispatch for kernels templated on <DT, OP>.
#define MSCCLPP_AMD_DISPATCH(dtype, op, FN, ...)                 \
  switch ((dtype) * 2 + (op)) {                                  \
    case kF16 * 2 + kSum: FN<kF16, kSum>(__VA_ARGS__); break;    \
    case kF16 * 2 + kMin: FN<kF16, kMin>(__VA_ARGS__); break;    \
    case kBF16 * 2 + kSum: FN<kBF16, kSum>(__VA_ARGS__); break;  \
    case kBF16 * 2 + kMin: FN<kBF16, kMin>(__VA_ARGS__); break;  \
    case kF32 * 2 + kSum: FN<kF32, kSum>(__VA_ARGS__); break;    \
    case kF32 * 2 + kMin: FN<kF32, kMin>(__VA_ARGS__); break;    \
    case kI32 * 2 + kSum: FN<kI32, kSum>(__VA_ARGS__); break;    \
    case kI32 * 2 + kMin: FN<kI32, kMin>(__VA_ARGS__); break;    \
    case kU32 * 2 + kSum: FN<kU32, kSum>(__VA_ARGS__); break;    \
    case kU32 * 2 + kMin: FN<kU32, kMin>(__VA_ARGS__); break;    \
    default: return 4; /* invalid argument */                    \
  }

// Both ops of one reduce type.
#define MSCCLPP_AMD_CASE2(DT, FN, ...)                      \
  case DT * 2 + kSum: FN<DT, kSum>(__VA_ARGS__); break;     \
  case DT * 2 + kMin: FN<DT, kMin>(__VA_ARGS__); break;

// As MSCCLPP_AMD_DISPATCH, plus the 1-byte reduce types: OCP FP8 and e4m3b15 with their
// accumulation types (dispatchFp8Accum, common.hpp:89-100) and uint8.
#define MSCCLPP_AMD_DISPATCH_ALL(dtype, op, FN, ...)     \
  switch ((dtype) * 2 + (op)) {                          \
    MSCCLPP_AMD_CASE2(kF16, FN, __VA_ARGS__)             \
    MSCCLPP_AMD_CASE2(kBF16, FN, __VA_ARGS__)            \
    MSCCLPP_AMD_CASE2(kF32, FN, __VA_ARGS__)             \
    MSCCLPP_AMD_CASE2(kI32, FN, __VA_ARGS__)             \
    MSCCLPP_AMD_CASE2(kU32, FN, __VA_ARGS__)             \
    MSCCLPP_AMD_CASE2(kE4M3, FN, __VA_ARGS__)            \
    MSCCLPP_AMD_CASE2(kE5M2, FN, __VA_ARGS__)            \
    MSCCLPP_AMD_CASE2(kE4M3AccF16, FN, __VA_ARGS__)      \
    MSCCLPP_AMD_CASE2(kE5M2AccF16, FN, __VA_ARGS__)      \
    MSCCLPP_AMD_CASE2(kE4M3AccF32, FN, __VA_ARGS__)      \
    MSCCLPP_AMD_CASE2(kE5M2AccF32, FN, __VA_ARGS__)      \
    MSCCLPP_AMD_CASE2(kU8, FN, __VA_ARGS__)              \
    MSCCLPP_AMD_CASE2(kB15, FN, __VA_ARGS__)             \
    MSCCLPP_AMD_CASE2(kB15AccF16, FN, __VA_ARGS__)       \
    MSCCLPP_AMD_CASE2(kB15AccF32, FN, __VA_ARGS__)       \
    default: return 4; /* invalid argument */            \
  }

}  // namespace mscclpp_amd
