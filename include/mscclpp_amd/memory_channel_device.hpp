// MemoryChannel device surface for gfx950: one-sided put / get / read / write, putPackets /
// unpackPackets (LL16 or LL8) and signal / wait over peer memory mapped through IPC.
//
// API shape follows include/mscclpp/memory_channel_device.hpp:15-224 and semaphore_device.hpp:61-135
// (same member names, argument order and meaning); every wait takes a time budget and reports
// timeouts through the device error word instead of asserting.  Stores into peer memory are
// system-scope write-through; polls of local memory written by peers are system-scope loads.
// The threaded helpers keep the reference's "thread tid of nthreads handles packets tid,
// tid + nthreads, ..." mapping, which is packet-major: consecutive lanes move consecutive 16-byte
// packets, so each wave instruction is one contiguous 1 KiB access.
#pragma once

#include "packet_device.hpp"

namespace mscclpp_amd {

struct MemoryDevice2DeviceSemaphoreDeviceHandle {
  uint64_t* inboundToken;          // local, written (added to) by the peer
  uint64_t* remoteInboundToken;    // the peer's inboundToken as mapped here
  uint64_t* expectedInboundToken;  // local wait counter

#if defined(__HIP__)
  // semaphore_device.hpp:84-90: prior memory operations complete before the peer sees the signal
  __device__ __forceinline__ void signal() { add_release_sys(remoteInboundToken, 1); }
  __device__ __forceinline__ void relaxedSignal() { add_relaxed_sys(remoteInboundToken, 1); }
  __device__ __forceinline__ bool poll() {
    const uint64_t want = __hip_atomic_load(expectedInboundToken, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
    if (ld_acquire_sys(inboundToken) >= want) {
      __hip_atomic_fetch_add(expectedInboundToken, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return true;
    }
    return false;
  }
  __device__ __forceinline__ bool wait(uint64_t budget, uint32_t* err) {
    const uint64_t want =
        __hip_atomic_fetch_add(expectedInboundToken, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
    SpinGuard g(budget);
    while (ld_relaxed_sys(inboundToken) < want) {
      if (g.expired()) {
        report_error(err, kErrSemaphoreTimeout);
        return false;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the invalidate completes before the barrier
    return true;
  }
  __device__ __forceinline__ bool relaxedWait(uint64_t budget, uint32_t* err) {
    const uint64_t want =
        __hip_atomic_fetch_add(expectedInboundToken, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
    SpinGuard g(budget);
    while (ld_relaxed_sys(inboundToken) < want) {
      if (g.expired()) {
        report_error(err, kErrSemaphoreTimeout);
        return false;
      }
    }
    return true;
  }
#endif
};

struct MemoryChannelDeviceHandle {
  MemoryDevice2DeviceSemaphoreDeviceHandle semaphore_;
  void* dst_;           // peer memory (mapped here)
  void* src_;           // local memory
  void* packetBuffer_;  // local packet buffer the peer puts packets into
  uint64_t budget_;     // spin budget in 10 ns ticks
  uint32_t* err_;       // device error word

#if defined(__HIP__)
  template <typename T>
  __device__ __forceinline__ T read(uint64_t index) {
    return *(reinterpret_cast<T*>(dst_) + index);
  }
  template <typename T>
  __device__ __forceinline__ void write(uint64_t index, const T& v) {
    *(reinterpret_cast<T*>(dst_) + index) = v;
  }

  // Threaded copy (copy_device.hpp:34-128): 16-byte vectors then 4-byte remainder; offsets and
  // sizes must be 4-byte aligned.  put writes peer memory write-through at system scope.
  __device__ __forceinline__ void put(uint64_t targetOffset, uint64_t originOffset, uint64_t bytes, uint32_t tid,
                                      uint32_t nthreads) {
    copySys(reinterpret_cast<char*>(dst_) + targetOffset, reinterpret_cast<const char*>(src_) + originOffset, bytes,
            tid, nthreads, true);
  }
  __device__ __forceinline__ void put(uint64_t offset, uint64_t bytes, uint32_t tid, uint32_t nthreads) {
    put(offset, offset, bytes, tid, nthreads);
  }
  __device__ __forceinline__ void get(uint64_t targetOffset, uint64_t originOffset, uint64_t bytes, uint32_t tid,
                                      uint32_t nthreads) {
    copySys(reinterpret_cast<char*>(src_) + targetOffset, reinterpret_cast<const char*>(dst_) + originOffset, bytes,
            tid, nthreads, false);
  }
  __device__ __forceinline__ void get(uint64_t offset, uint64_t bytes, uint32_t tid, uint32_t nthreads) {
    get(offset, offset, bytes, tid, nthreads);
  }

  // putPackets<LL16>: 8 payload bytes per packet; putPackets<LL8>: 4 (memory_channel_device.hpp:154-168)
  template <typename PacketType = LL16Packet>
  __device__ __forceinline__ void putPackets(uint64_t targetOffset, uint64_t originOffset, uint64_t bytes,
                                             uint32_t tid, uint32_t nthreads, uint32_t flag) {
    char* dst = reinterpret_cast<char*>(dst_) + targetOffset;
    const uint32_t* s = reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(src_) + originOffset);
    if constexpr (sizeof(PacketType) == 16) {
      const auto r = make_rsrc(dst);
      for (uint64_t i = tid; i < bytes / 8; i += nthreads)
        store16<kSystem>(r, (uint32_t)(i * 16), LL16Packet::make(s[2 * i], s[2 * i + 1], flag));
    } else {
      const auto r = make_rsrc(dst);
      for (uint64_t i = tid; i < bytes / 4; i += nthreads) store8<kSystem>(r, (uint32_t)(i * 8), u32x2{s[i], flag});
    }
  }
  template <typename PacketType = LL16Packet>
  __device__ __forceinline__ void putPackets(uint64_t offset, uint64_t bytes, uint32_t tid, uint32_t nthreads,
                                             uint32_t flag) {
    putPackets<PacketType>(offset, offset, bytes, tid, nthreads, flag);
  }
  // unpackPackets: poll the local packet buffer, write the payload into local memory (:178-215)
  template <typename PacketType = LL16Packet>
  __device__ __forceinline__ void unpackPackets(uint64_t targetOffset, uint64_t originOffset, uint64_t bytes,
                                                uint32_t tid, uint32_t nthreads, uint32_t flag) {
    uint32_t* d = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(src_) + originOffset);
    const char* pk = reinterpret_cast<const char*>(packetBuffer_) + targetOffset;
    const auto r = make_rsrc(pk);
    if constexpr (sizeof(PacketType) == 16) {
      for (uint64_t i = tid; i < bytes / 8; i += nthreads) {
        u32x4 v = load16<kSystem>(r, (uint32_t)(i * 16));
        if (!LL16Packet::ready(v, flag)) {
          SpinGuard g(budget_);
          do {
            v = load16<kSystem>(r, (uint32_t)(i * 16));
            if (g.expired()) {
              report_error(err_, kErrPacketTimeout);
              break;
            }
          } while (!LL16Packet::ready(v, flag));
        }
        d[2 * i] = v.x;
        d[2 * i + 1] = v.z;
      }
    } else {
      for (uint64_t i = tid; i < bytes / 4; i += nthreads) {
        u32x2 v = load8<kSystem>(r, (uint32_t)(i * 8));
        if (v.y != flag) {
          SpinGuard g(budget_);
          do {
            v = load8<kSystem>(r, (uint32_t)(i * 8));
            if (g.expired()) {
              report_error(err_, kErrPacketTimeout);
              break;
            }
          } while (v.y != flag);
        }
        d[i] = v.x;
      }
    }
  }
  template <typename PacketType = LL16Packet>
  __device__ __forceinline__ void unpackPackets(uint64_t offset, uint64_t bytes, uint32_t tid, uint32_t nthreads,
                                                uint32_t flag) {
    unpackPackets<PacketType>(offset, offset, bytes, tid, nthreads, flag);
  }

  __device__ __forceinline__ void signal() { semaphore_.signal(); }
  __device__ __forceinline__ void relaxedSignal() { semaphore_.relaxedSignal(); }
  __device__ __forceinline__ bool poll() { return semaphore_.poll(); }
  __device__ __forceinline__ void wait() { semaphore_.wait(budget_, err_); }
  __device__ __forceinline__ void relaxedWait() { semaphore_.relaxedWait(budget_, err_); }

 private:
  __device__ __forceinline__ static void copySys(char* dst, const char* src, uint64_t bytes, uint32_t tid,
                                                 uint32_t nthreads, bool remoteDst) {
    const auto rd = make_rsrc(dst);
    const auto rs = make_rsrc(src);
    const uint64_t n16 = bytes / 16;
    for (uint64_t i = tid; i < n16; i += nthreads) {
      const u32x4 v = remoteDst ? load16<kPlain>(rs, (uint32_t)(i * 16)) : load16<kSystem>(rs, (uint32_t)(i * 16));
      if (remoteDst)
        store16<kSystem>(rd, (uint32_t)(i * 16), v);
      else
        store16<kPlain>(rd, (uint32_t)(i * 16), v);
    }
    for (uint64_t i = n16 * 4 + tid; i < bytes / 4; i += nthreads) {
      const uint32_t v = remoteDst ? load4<kPlain>(rs, (uint32_t)(i * 4)) : load4<kSystem>(rs, (uint32_t)(i * 4));
      if (remoteDst)
        store4<kSystem>(rd, (uint32_t)(i * 4), v);
      else
        store4<kPlain>(rd, (uint32_t)(i * 4), v);
    }
  }
#endif
};

}  // namespace mscclpp_amd
