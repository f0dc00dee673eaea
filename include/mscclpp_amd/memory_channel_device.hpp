// MemoryChannel device surface for gfx950: one-sided put / get / read / write, putPackets /
// unpackPacket(s) (LL16 or LL8) and signal / wait over peer memory mapped through IPC.
//
// Spellings, argument order and meaning follow include/mscclpp/memory_channel_device.hpp:15-224
// (BaseMemoryChannelDeviceHandle { semaphore_ }, MemoryChannelDeviceHandle { dst_, src_,
// packetBuffer_ }), so a kernel written against the reference compiles here after a namespace
// change.  What differs is underneath: stores into peer memory (put, putPackets) are 16-byte
// system-scope write-through buffer stores, loads of peer memory (get) are system-scope, and every
// wait is bounded by the semaphore handle's wall-clock budget and reports through its error word
// instead of spinning forever.  The threaded helpers keep the reference's "thread tid of nthreads
// handles elements tid, tid + nthreads, ..." mapping, which is packet-major: consecutive lanes move
// consecutive 16-byte packets, so each wave instruction is one contiguous 1 KiB access.
#pragma once

#include "copy_device.hpp"
#include "semaphore_device.hpp"

namespace mscclpp_amd {

// memory_channel_device.hpp:15-54
struct BaseMemoryChannelDeviceHandle {
  MemoryDevice2DeviceSemaphoreDeviceHandle semaphore_;

  BaseMemoryChannelDeviceHandle() = default;
  __host__ __device__ BaseMemoryChannelDeviceHandle(MemoryDevice2DeviceSemaphoreDeviceHandle semaphore)
      : semaphore_(semaphore) {}

#if defined(__HIP__)
  __device__ __forceinline__ void signal() { semaphore_.signal(); }
  __device__ __forceinline__ void relaxedSignal() { semaphore_.relaxedSignal(); }
  __device__ __forceinline__ bool poll() { return semaphore_.poll(); }
  __device__ __forceinline__ void wait(int64_t maxSpinCount = 10000000) { semaphore_.wait(maxSpinCount); }
  __device__ __forceinline__ void relaxedWait(int64_t maxSpinCount = 10000000) {
    semaphore_.relaxedWait(maxSpinCount);
  }
#endif
};

// memory_channel_device.hpp:56-224
struct MemoryChannelDeviceHandle : public BaseMemoryChannelDeviceHandle {
  void* dst_;           // peer memory (mapped here)
  void* src_;           // local memory
  void* packetBuffer_;  // local packet buffer the peer puts packets into (may be null)

  MemoryChannelDeviceHandle() = default;
  __host__ __device__ MemoryChannelDeviceHandle(MemoryDevice2DeviceSemaphoreDeviceHandle semaphore, void* dst,
                                                void* src, void* packetBuffer)
      : BaseMemoryChannelDeviceHandle(semaphore), dst_(dst), src_(src), packetBuffer_(packetBuffer) {}

#if defined(__HIP__)
  template <typename T>
  __device__ __forceinline__ T read(uint64_t index) {
    return *(reinterpret_cast<T*>(dst_) + index);
  }
  template <typename T>
  __device__ __forceinline__ void write(uint64_t index, const T& v) {
    *(reinterpret_cast<T*>(dst_) + index) = v;
  }

  // Threaded copy local -> peer (copy_device.hpp:34-128 semantics: 4-byte head, Alignment-sized
  // body, 4-byte tail; offsets and sizes 4-byte aligned).  The peer side is written through at
  // system scope, 16 bytes per lane where the alignment allows; each lane's stores have completed
  // when put returns.
  template <int Alignment = 16, bool CopyRemainder = true>
  __device__ __forceinline__ void put(uint64_t targetOffset, uint64_t originOffset, uint64_t originBytes,
                                     uint32_t threadId, uint32_t numThreads) {
    copySys<Alignment, CopyRemainder, true>(reinterpret_cast<char*>(dst_) + targetOffset,
                                            reinterpret_cast<const char*>(src_) + originOffset, originBytes,
                                            threadId, numThreads);
  }
  template <int Alignment = 16, bool CopyRemainder = true>
  __device__ __forceinline__ void put(uint64_t offset, uint64_t originBytes, uint32_t threadId, uint32_t numThreads) {
    put<Alignment, CopyRemainder>(offset, offset, originBytes, threadId, numThreads);
  }
  // Threaded copy peer -> local (the peer side is read through at system scope).
  template <int Alignment = 16, bool CopyRemainder = true>
  __device__ __forceinline__ void get(uint64_t targetOffset, uint64_t originOffset, uint64_t originBytes,
                                     uint32_t threadId, uint32_t numThreads) {
    copySys<Alignment, CopyRemainder, false>(reinterpret_cast<char*>(src_) + targetOffset,
                                             reinterpret_cast<const char*>(dst_) + originOffset, originBytes,
                                             threadId, numThreads);
  }
  template <int Alignment = 16, bool CopyRemainder = true>
  __device__ __forceinline__ void get(uint64_t offset, uint64_t originBytes, uint32_t threadId, uint32_t numThreads) {
    get<Alignment, CopyRemainder>(offset, offset, originBytes, threadId, numThreads);
  }

  // putPackets<LL16>: 8 payload bytes per packet; putPackets<LL8>: 4 (memory_channel_device.hpp:154-168)
  template <typename PacketType = LL16Packet>
  __device__ __forceinline__ void putPackets(uint64_t targetOffset, uint64_t originOffset, uint64_t originBytes,
                                             uint32_t threadId, uint32_t numThreads, uint32_t flag) {
    static_assert(sizeof(PacketType) == 16 || sizeof(PacketType) == 8, "Unsupported packet type");
    char* dst = reinterpret_cast<char*>(dst_) + targetOffset;
    const uint32_t* s = reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(src_) + originOffset);
    if constexpr (sizeof(PacketType) == 16) {
      for_each_strided<16>(originBytes / 8, threadId, numThreads, [&](uint64_t i, uint64_t w0, uint32_t off) {
        store16<kSystem>(make_rsrc(dst + w0 * 16), off, LL16Packet::make(s[2 * i], s[2 * i + 1], flag));
      });
    } else {
      for_each_strided<8>(originBytes / 4, threadId, numThreads, [&](uint64_t i, uint64_t w0, uint32_t off) {
        store8<kSystem>(make_rsrc(dst + w0 * 8), off, u32x2{s[i], flag});
      });
    }
  }
  template <typename PacketType = LL16Packet>
  __device__ __forceinline__ void putPackets(uint64_t offset, uint64_t originBytes, uint32_t threadId,
                                             uint32_t numThreads, uint32_t flag) {
    putPackets<PacketType>(offset, offset, originBytes, threadId, numThreads, flag);
  }

  // One packet of the local packet buffer (memory_channel_device.hpp:178-182): uint2 for LL16,
  // uint32_t for LL8.
  template <typename PacketType = LL16Packet>
  __device__ __forceinline__ auto unpackPacket(uint64_t index, uint32_t flag, int64_t maxSpinCount = -1) {
    return reinterpret_cast<const PacketType*>(packetBuffer_)[index].read(flag, maxSpinCount);
  }

  // Poll the local packet buffer, write the payload into local memory (:198-215).  Each lane
  // polls whole packets with one 16-byte (LL16) / 8-byte (LL8) system-scope load.
  template <typename PacketType = LL16Packet>
  __device__ __forceinline__ void unpackPackets(uint64_t targetOffset, uint64_t originOffset, uint64_t originBytes,
                                                uint32_t threadId, uint32_t numThreads, uint32_t flag,
                                                int64_t maxSpinCount = -1) {
    static_assert(sizeof(PacketType) == 16 || sizeof(PacketType) == 8, "Unsupported packet type");
    (void)maxSpinCount;
    uint32_t* d = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(src_) + originOffset);
    const char* pk = reinterpret_cast<const char*>(packetBuffer_) + targetOffset;
    const uint64_t budget = semaphore_.budget ? semaphore_.budget : kDefaultSpinTicks;
    if constexpr (sizeof(PacketType) == 16) {
      for_each_strided<16>(originBytes / 8, threadId, numThreads, [&](uint64_t i, uint64_t w0, uint32_t off) {
        const auto r = make_rsrc(pk + w0 * 16);
        u32x4 v = load16<kSystem>(r, off);
        if (!LL16Packet::ready(v, flag)) {
          SpinGuard g(budget);
          do {
            v = load16<kSystem>(r, off);
            if (g.expired()) {
              report_packet_timeout(semaphore_.err, flag, targetOffset + i * 16, v.y != flag ? v.y : v.w);
              break;
            }
          } while (!LL16Packet::ready(v, flag));
        }
        d[2 * i] = v.x;
        d[2 * i + 1] = v.z;
      });
    } else {
      for_each_strided<8>(originBytes / 4, threadId, numThreads, [&](uint64_t i, uint64_t w0, uint32_t off) {
        const auto r = make_rsrc(pk + w0 * 8);
        u32x2 v = load8<kSystem>(r, off);
        if (v.y != flag) {
          SpinGuard g(budget);
          do {
            v = load8<kSystem>(r, off);
            if (g.expired()) {
              report_packet_timeout(semaphore_.err, flag, targetOffset + i * 8, v.y);
              break;
            }
          } while (v.y != flag);
        }
        d[i] = v.x;
      });
    }
  }
  template <typename PacketType = LL16Packet>
  __device__ __forceinline__ void unpackPackets(uint64_t offset, uint64_t originBytes, uint32_t threadId,
                                                uint32_t numThreads, uint32_t flag, int64_t maxSpinCount = -1) {
    unpackPackets<PacketType>(offset, offset, originBytes, threadId, numThreads, flag, maxSpinCount);
  }

 private:
  // Threaded copy with the remote side at system scope: 4-byte head to the first Alignment boundary
  // of dst, Alignment-sized body (16 B: one dwordx4 per lane), 4-byte tail.
  template <int Alignment, bool CopyRemainder, bool RemoteDst>
  __device__ __forceinline__ static void copySys(char* dst, const char* src, uint64_t bytes, uint32_t tid,
                                                 uint32_t nthreads) {
    static_assert(Alignment == 4 || Alignment == 8 || Alignment == 16, "Unsupported alignment");
    constexpr int kRemote = kSystem, kLocal = kPlain;
    const uint64_t numInt = bytes / 4;
    const uintptr_t d = reinterpret_cast<uintptr_t>(dst);
    uint64_t head = ((d + Alignment - 1) / Alignment * Alignment - d) / 4;
    if (head > numInt) head = numInt;
    auto copy4 = [&](uint64_t from, uint64_t n) {
      for_each_strided<4>(n, tid, nthreads, [&](uint64_t, uint64_t w0, uint32_t off) {
        const auto rd = make_rsrc(dst + (from + w0) * 4);
        const auto rs = make_rsrc(src + (from + w0) * 4);
        const uint32_t v = RemoteDst ? load4<kLocal>(rs, off) : load4<kRemote>(rs, off);
        if (RemoteDst)
          store4<kRemote>(rd, off, v);
        else
          store4<kLocal>(rd, off, v);
      });
    };
    if (CopyRemainder) copy4(0, head);
    constexpr uint64_t kIntPer = Alignment / 4;
    const uint64_t nElem = (numInt - head) / kIntPer;
    for_each_strided<Alignment>(nElem, tid, nthreads, [&](uint64_t, uint64_t w0, uint32_t off) {
      const auto rd = make_rsrc(dst + head * 4 + w0 * Alignment);
      const auto rs = make_rsrc(src + head * 4 + w0 * Alignment);
      if constexpr (Alignment == 16) {
        const u32x4 v = RemoteDst ? load16<kLocal>(rs, off) : load16<kRemote>(rs, off);
        if (RemoteDst)
          store16<kRemote>(rd, off, v);
        else
          store16<kLocal>(rd, off, v);
      } else if constexpr (Alignment == 8) {
        const u32x2 v = RemoteDst ? load8<kLocal>(rs, off) : load8<kRemote>(rs, off);
        if (RemoteDst)
          store8<kRemote>(rd, off, v);
        else
          store8<kLocal>(rd, off, v);
      } else {
        const uint32_t v = RemoteDst ? load4<kLocal>(rs, off) : load4<kRemote>(rs, off);
        if (RemoteDst)
          store4<kRemote>(rd, off, v);
        else
          store4<kLocal>(rd, off, v);
      }
    });
    if (CopyRemainder && kIntPer > 1) copy4(head + nElem * kIntPer, numInt - head - nElem * kIntPer);
    // this lane's copies are complete when it returns, so a workgroup barrier followed by one
    // lane's signal() publishes the whole workgroup's put (or its get's data to the other waves)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
#endif
};

}  // namespace mscclpp_amd
