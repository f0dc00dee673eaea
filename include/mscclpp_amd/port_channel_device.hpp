// Host-proxy (PortChannel) device primitives for gfx950: ProxyTrigger, the GPU->host trigger FIFO,
// Host2Device semaphores and the PortChannel put / signal / flush / wait surface.
//
// Behaviour follows the reference:
//   ProxyTrigger bit layout        include/mscclpp/fifo_device.hpp:35-92 (fst = srcOffset<<32 | size;
//                                  snd = dstOffset | srcId<<32 | dstId<<41 | type<<50 | semId<<53 | commit<<63)
//   FifoDeviceHandle::push / sync  fifo_device.hpp:103-183 (commit bit = lap parity, :120)
//   Host2DeviceSemaphore wait      semaphore_device.hpp:17-58
//   PortChannel put/signal/flush   port_channel_device.hpp:33-195
// gfx950 specifics: the trigger payload word is published with a relaxed system-scope store and the
// commit word with a release system-scope store (the FIFO lives in host-pinned, device-mapped
// memory); every wait is time-bounded and reports through the device error word.
#pragma once

#include "device.hpp"

namespace mscclpp_amd {

using TriggerType = uint64_t;
constexpr TriggerType kTriggerData = 0x1;  // data transfer
constexpr TriggerType kTriggerFlag = 0x2;  // signal
constexpr TriggerType kTriggerSync = 0x4;  // flush

union alignas(16) ProxyTrigger {
  struct {
    uint64_t fst;
    uint64_t snd;
  };
  struct {
    uint64_t size : 32;
    uint64_t srcOffset : 32;
    uint64_t dstOffset : 32;
    uint64_t srcMemoryId : 9;
    uint64_t dstMemoryId : 9;
    uint64_t type : 3;
    uint64_t semaphoreId : 10;
    uint64_t reserved : 1;  // FIFO commit bit
  } fields;
};
static_assert(sizeof(ProxyTrigger) == 16, "ProxyTrigger must be two 64-bit words");

__host__ __device__ inline ProxyTrigger makeTrigger(TriggerType type, uint32_t dstId, uint64_t dstOffset, uint32_t srcId,
                                                    uint64_t srcOffset, uint64_t bytes, uint32_t semaphoreId) {
  const uint64_t m32 = 0xffffffffull, m9 = 0x1ffull, m3 = 0x7ull, m10 = 0x3ffull;
  ProxyTrigger t;
  t.fst = ((srcOffset & m32) << 32) + (bytes & m32);
  t.snd = ((((((((semaphoreId & m10) << 3) + (type & m3)) << 9) + (dstId & m9)) << 9) + (srcId & m9)) << 32) +
          (dstOffset & m32);
  return t;
}

struct FifoDeviceHandle {
  ProxyTrigger* triggers;  // host-pinned, device-mapped ring
  uint64_t* head;          // device memory
  uint64_t* tail;          // host-pinned, device-mapped (written by the proxy)
  uint64_t* tailCache;     // device memory
  int size;                // power of two
  uint64_t sizeMask;
  uint64_t sizeShift;

#if defined(__HIP__)
  // Wait until the trigger at `pos` has been popped by the proxy.
  __device__ __forceinline__ bool sync(uint64_t pos, uint64_t budget, uint32_t* err) {
    SpinGuard g(budget);
    uint64_t v;
    while (pos >= (v = ld_acquire_sys(tail))) {
      if (g.expired()) {
        report_error(err, kErrFifoTimeout);
        return false;
      }
    }
    __hip_atomic_store(tailCache, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
  }
  __device__ __forceinline__ bool poll(uint64_t pos) {
    uint64_t v = ld_acquire_sys(tail);
    if (pos < v) {
      __hip_atomic_store(tailCache, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return true;
    }
    return false;
  }
  // Push a trigger; returns its FIFO position (the reference's push return value).
  __device__ __forceinline__ uint64_t push(ProxyTrigger t, uint64_t budget, uint32_t* err) {
    const uint64_t pos = __hip_atomic_fetch_add(head, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // the slot's previous occupant must have been consumed (lap parity alone cannot tell)
    if (pos >= (uint64_t)size + __hip_atomic_load(tailCache, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      sync(pos - size, budget, err);
    t.fields.reserved = ((pos >> sizeShift) & 1ull) ^ 1ull;  // lap 0 writes 1 (fifo_device.hpp:120)
    ProxyTrigger* slot = &triggers[pos & sizeMask];
    st_relaxed_sys(&slot->fst, t.fst);
    st_release_sys(&slot->snd, t.snd);  // commit word last: the payload is visible with it
    return pos;
  }
#endif
};

struct Host2DeviceSemaphoreDeviceHandle {
  uint64_t* inboundToken;          // device memory, written by the peer's proxy (hipMemcpyAsync)
  uint64_t* expectedInboundToken;  // device memory

#if defined(__HIP__)
  __device__ __forceinline__ bool poll() {
    const uint64_t want = *expectedInboundToken + 1;
    if (ld_acquire_sys(inboundToken) >= want) {
      *expectedInboundToken = want;
      return true;
    }
    return false;
  }
  __device__ __forceinline__ bool wait(uint64_t budget, uint32_t* err) {
    const uint64_t want = *expectedInboundToken + 1;
    *expectedInboundToken = want;
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
#endif
};

struct PortChannelDeviceHandle {
  uint32_t semaphoreId;
  uint32_t dst;  // MemoryId of the destination region (peer)
  uint32_t src;  // MemoryId of the source region (local)
  uint32_t pad;
  Host2DeviceSemaphoreDeviceHandle semaphore;
  FifoDeviceHandle fifo;
  uint64_t* flushDonePos;  // host-pinned: one past the highest FIFO position whose flush completed
  uint64_t budget;         // spin budget (10 ns ticks)
  uint32_t* err;

#if defined(__HIP__)
  __device__ __forceinline__ void put(uint64_t dstOffset, uint64_t srcOffset, uint64_t bytes) {
    fifo.push(makeTrigger(kTriggerData, dst, dstOffset, src, srcOffset, bytes, semaphoreId), budget, err);
  }
  __device__ __forceinline__ void put(uint64_t offset, uint64_t bytes) { put(offset, offset, bytes); }
  __device__ __forceinline__ void signal() {
    fifo.push(makeTrigger(kTriggerFlag, 0, 0, 0, 0, 0, semaphoreId), budget, err);
  }
  __device__ __forceinline__ void putWithSignal(uint64_t dstOffset, uint64_t srcOffset, uint64_t bytes) {
    fifo.push(makeTrigger(kTriggerData | kTriggerFlag, dst, dstOffset, src, srcOffset, bytes, semaphoreId), budget, err);
  }
  __device__ __forceinline__ void waitFlush(uint64_t pos) {
    SpinGuard g(budget);
    while (ld_acquire_sys(flushDonePos) <= pos) {
      if (g.expired()) {
        report_error(err, kErrFifoTimeout);
        return;
      }
    }
  }
  __device__ __forceinline__ void putWithSignalAndFlush(uint64_t dstOffset, uint64_t srcOffset, uint64_t bytes) {
    waitFlush(fifo.push(
        makeTrigger(kTriggerData | kTriggerFlag | kTriggerSync, dst, dstOffset, src, srcOffset, bytes, semaphoreId),
        budget, err));
  }
  __device__ __forceinline__ void flush() {
    waitFlush(fifo.push(makeTrigger(kTriggerSync, 0, 0, 0, 0, 0, semaphoreId), budget, err));
  }
  __device__ __forceinline__ bool poll() { return semaphore.poll(); }
  __device__ __forceinline__ void wait() { semaphore.wait(budget, err); }
#endif
};

}  // namespace mscclpp_amd
