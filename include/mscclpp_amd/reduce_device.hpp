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

// Reduce types.  0..4 accumulate in the element type.  The FP8 codes (OCP e4m3 / e5m2, the
// gfx950 hardware formats) carry the accumulation type of calVectorAccum<T, AccumT, Op>
// (reduce_kernel.hpp:171-189, dispatchFp8Accum common.hpp:89-100): T, half or float.
enum DType : int {
  kF16 = 0, kBF16 = 1, kF32 = 2, kI32 = 3, kU32 = 4,
  kE4M3 = 5, kE5M2 = 6,              // AccumT = T
  kE4M3AccF16 = 7, kE5M2AccF16 = 8,  // AccumT = half
  kE4M3AccF32 = 9, kE5M2AccF32 = 10  // AccumT = float
};
enum ROp : int { kSum = 0, kMin = 1 };

__host__ __device__ constexpr bool is_fp8(int dt) { return dt >= kE4M3 && dt <= kE5M2AccF32; }
__host__ __device__ constexpr bool is_e5m2(int dt) { return dt == kE5M2 || dt == kE5M2AccF16 || dt == kE5M2AccF32; }
__host__ __device__ constexpr int elem_bytes(int dt) { return (dt == kF16 || dt == kBF16) ? 2 : (is_fp8(dt) ? 1 : 4); }

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

// Word accumulator: up(word) -> acc; add(acc, word) -> acc; down(acc) -> word.
template <int DT, int OP, int KIND = (DT == kE4M3AccF16 || DT == kE5M2AccF16) ? 1
                                     : ((DT == kE4M3AccF32 || DT == kE5M2AccF32) ? 2 : 0)>
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
  } else if constexpr (is_fp8(DT)) {
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

// As MSCCLPP_AMD_DISPATCH, plus the FP8 reduce types (dispatchFp8Accum, common.hpp:89-100).
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
    default: return 4; /* invalid argument */            \
  }

}  // namespace mscclpp_amd
