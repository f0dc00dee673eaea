// Threaded copies and packet copies for gfx950, with the reference's spellings
// (include/mscclpp/copy_device.hpp:34-232):
//   copy<Alignment, CopyRemainder>(dst, src, bytes, threadId, numThreads)
//   copyToPackets<PacketType>(target, origin, originBytes, threadId, numThreads, flag)
//   copyFromPackets<PacketType>(origin, target, originBytes, threadId, numThreads, flag, maxSpinCount)
//   write<T>(dst, index, v) / read<T>(src, index)
// "thread `threadId` of `numThreads` handles elements threadId, threadId + numThreads, ..." as in the
// reference, so consecutive lanes touch consecutive elements: every wave instruction is one
// contiguous access.  Packet writes are one 16-byte (LL16) or 8-byte (LL8) system-scope store per
// packet; packet reads spin with a wall-clock bound (device.hpp: kDefaultSpinTicks).
#pragma once

#include "packet_device.hpp"

namespace mscclpp_amd {

namespace detail {
template <typename T>
__device__ __forceinline__ void copyElems(T* dst, const T* src, uint64_t numElems, uint32_t threadId,
                                          uint32_t numThreads) {
  for (uint64_t i = threadId; i < numElems; i += numThreads) {
    const T reg = src[i];
    dst[i] = reg;
  }
}
}  // namespace detail

// copy_device.hpp:68-92: 4-byte head up to the first T-aligned address, T-sized body, 4-byte tail.
// The misalignment of src and dst to sizeof(T) must be the same multiple of 4 bytes; bytes % 4 == 0.
template <typename T, bool CopyRemainder = true>
__device__ __forceinline__ void copyHelper(void* dst, const void* src, uint64_t bytes, uint32_t threadId,
                                           uint32_t numThreads) {
  const uintptr_t d = reinterpret_cast<uintptr_t>(dst), s = reinterpret_cast<uintptr_t>(src);
  const uint64_t numInt = bytes / 4;
  const uintptr_t dAligned = (d + sizeof(T) - 1) / sizeof(T) * sizeof(T);
  uint64_t head = (dAligned - d) / 4;
  if (head > numInt) head = numInt;
  if constexpr (CopyRemainder) detail::copyElems<int>((int*)dst, (const int*)src, head, threadId, numThreads);
  constexpr uint64_t kIntPerElem = sizeof(T) / 4;
  const uint64_t nElem = (numInt - head) / kIntPerElem;
  detail::copyElems<T>(reinterpret_cast<T*>(d + head * 4), reinterpret_cast<const T*>(s + head * 4), nElem, threadId,
                       numThreads);
  if constexpr (CopyRemainder && kIntPerElem > 1) {
    const uint64_t done = head + nElem * kIntPerElem;
    detail::copyElems<int>((int*)dst + done, (const int*)src + done, numInt - done, threadId, numThreads);
  }
}

template <int Alignment = 16, bool CopyRemainder = true>
__device__ __forceinline__ void copy(void* dst, const void* src, uint64_t bytes, uint32_t threadId,
                                     uint32_t numThreads) {
  static_assert(Alignment == 4 || Alignment == 8 || Alignment == 16, "Unsupported alignment");
  if constexpr (Alignment == 4)
    copyHelper<int, CopyRemainder>(dst, src, bytes, threadId, numThreads);
  else if constexpr (Alignment == 8)
    copyHelper<long long, CopyRemainder>(dst, src, bytes, threadId, numThreads);
  else
    copyHelper<u32x4, CopyRemainder>(dst, src, bytes, threadId, numThreads);
}

template <typename T>
__device__ __forceinline__ void write(void* dst, uint64_t index, const T& v) {
  *(reinterpret_cast<T*>(dst) + index) = v;
}
template <typename T>
__device__ __forceinline__ T read(void* src, uint64_t index) {
  return *(reinterpret_cast<T*>(src) + index);
}

// copy_device.hpp:156-184: originBytes of payload -> packets (LL16: 8 B per packet, LL8: 4 B).
template <typename PacketType = LL16Packet>
__device__ __forceinline__ void copyToPackets(void* targetPtr, const void* originPtr, uint64_t originBytes,
                                              uint32_t threadId, uint32_t numThreads, uint32_t flag) {
  static_assert(sizeof(PacketType) == 16 || sizeof(PacketType) == 8, "Unsupported packet type");
  if constexpr (sizeof(PacketType) == 16)
    copyToPacketsLL16(targetPtr, originPtr, originBytes, threadId, numThreads, flag);
  else
    copyToPacketsLL8(targetPtr, originPtr, originBytes, threadId, numThreads, flag);
}

// copy_device.hpp:201-232: packets -> originBytes of payload, each packet polled until its flag(s)
// match.  maxSpinCount: accepted, see device.hpp; each wait is bounded by kDefaultSpinTicks.
template <typename PacketType = LL16Packet>
__device__ __forceinline__ void copyFromPackets(void* originPtr, const void* targetPtr, uint64_t originBytes,
                                                uint32_t threadId, uint32_t numThreads, uint32_t flag,
                                                int64_t maxSpinCount = -1) {
  static_assert(sizeof(PacketType) == 16 || sizeof(PacketType) == 8, "Unsupported packet type");
  const PacketType* pk = reinterpret_cast<const PacketType*>(targetPtr);
  if constexpr (sizeof(PacketType) == 16) {
    uint2* o = reinterpret_cast<uint2*>(originPtr);
    for (uint64_t i = threadId; i < originBytes / 8; i += numThreads) o[i] = pk[i].read(flag, maxSpinCount);
  } else {
    uint32_t* o = reinterpret_cast<uint32_t*>(originPtr);
    for (uint64_t i = threadId; i < originBytes / 4; i += numThreads) o[i] = pk[i].read(flag, maxSpinCount);
  }
}

}  // namespace mscclpp_amd
