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

enum DType : int { kF16 = 0, kBF16 = 1, kF32 = 2, kI32 = 3, kU32 = 4 };
enum ROp : int { kSum = 0, kMin = 1 };

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

template <int DT, int OP>
__device__ __forceinline__ uint32_t reduce_word(uint32_t acc, uint32_t val) {
  if constexpr (OP == kSum) {
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

}  // namespace mscclpp_amd
