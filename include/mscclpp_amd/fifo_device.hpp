// GPU -> host trigger FIFO for gfx950 (include/mscclpp/fifo_device.hpp:35-183).
//
// ProxyTrigger has the reference's bit layout (fst = srcOffset << 32 | size; snd = dstOffset |
// srcMemoryId << 32 | dstMemoryId << 41 | type << 50 | semaphoreId << 53 | commit << 63,
// fifo_device.hpp:35-92) and FifoDeviceHandle the reference's fields and push / poll / sync.  The
// commit bit of a slot is the lap parity of its position (fifo_device.hpp:118-120).  The payload word
// is published with a relaxed system-scope store and the commit word after it with a release
// system-scope store (the ring lives in host-pinned, device-mapped memory).  Two fields are this
// library's: `budget` bounds the wait for a free slot in wall-clock ticks, and `err` receives
// kErrFifoTimeout when it runs out.
#pragma once

#include "device.hpp"

namespace mscclpp_amd {

using TriggerType = uint64_t;
constexpr TriggerType TriggerData = 0x1;  // data transfer     (fifo_device.hpp:20-29)
constexpr TriggerType TriggerFlag = 0x2;  // signal
constexpr TriggerType TriggerSync = 0x4;  // flush
constexpr TriggerType kTriggerData = TriggerData;
constexpr TriggerType kTriggerFlag = TriggerFlag;
constexpr TriggerType kTriggerSync = TriggerSync;

constexpr unsigned int TriggerBitsSize = 32;
constexpr unsigned int TriggerBitsOffset = 32;
constexpr unsigned int TriggerBitsMemoryId = 9;
constexpr unsigned int TriggerBitsType = 3;
constexpr unsigned int TriggerBitsSemaphoreId = 10;

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

  ProxyTrigger() = default;
  // fifo_device.hpp:75-92
  __host__ __device__ ProxyTrigger(TriggerType type, uint32_t dstId, uint64_t dstOffset, uint32_t srcId,
                                   uint64_t srcOffset, uint64_t bytes, uint32_t semaphoreId) {
    const uint64_t m32 = 0xffffffffull, m9 = 0x1ffull, m3 = 0x7ull, m10 = 0x3ffull;
    fst = ((srcOffset & m32) << 32) + (bytes & m32);
    snd = ((((((((semaphoreId & m10) << 3) + (type & m3)) << 9) + (dstId & m9)) << 9) + (srcId & m9)) << 32) +
          (dstOffset & m32);
  }
};
static_assert(sizeof(ProxyTrigger) == 16, "ProxyTrigger must be two 64-bit words");

__host__ __device__ inline ProxyTrigger makeTrigger(TriggerType type, uint32_t dstId, uint64_t dstOffset, uint32_t srcId,
                                                    uint64_t srcOffset, uint64_t bytes, uint32_t semaphoreId) {
  return ProxyTrigger(type, dstId, dstOffset, srcId, srcOffset, bytes, semaphoreId);
}

struct FifoDeviceHandle {
  ProxyTrigger* triggers;  // host-pinned, device-mapped ring
  uint64_t* head;          // device memory
  uint64_t* tail;          // host-pinned, device-mapped (written by the proxy)
  uint64_t* tailCache;     // device memory
  int size;                // power of two
  uint64_t sizeMask;       // size - 1
  uint64_t sizeShift;      // log2(size)
  uint64_t budget;         // wall-clock bound of the waits (10 ns ticks; 0 = kDefaultSpinTicks)
  uint32_t* err;           // device error word (may be null)

#if defined(__HIP__)
  // Wait until the trigger pushed at `fifoHead` has been popped by the proxy (fifo_device.hpp:159-166).
  __device__ __forceinline__ void sync(uint64_t fifoHead, int64_t maxSpinCount = 1000000) {
    (void)maxSpinCount;
    SpinGuard g(budget ? budget : kDefaultSpinTicks);
    uint64_t v;
    while (fifoHead >= (v = ld_relaxed_sys(tail))) {
      if (g.expired()) {
        report_error(err, kErrFifoTimeout);
        return;
      }
    }
    acquire_sys();
    __hip_atomic_store(tailCache, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __device__ __forceinline__ bool poll(uint64_t fifoHead) {
    const uint64_t v = ld_acquire_sys(tail);
    if (fifoHead < v) {
      __hip_atomic_store(tailCache, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return true;
    }
    return false;
  }
  // Push a trigger; returns its FIFO position (fifo_device.hpp:109-141).
  __device__ __forceinline__ uint64_t push(ProxyTrigger trigger, int64_t maxSpinCount = 1000000) {
    const uint64_t pos = __hip_atomic_fetch_add(head, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // the slot's previous occupant must have been consumed (lap parity alone cannot tell)
    if (pos >= (uint64_t)size + __hip_atomic_load(tailCache, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      sync(pos - size, maxSpinCount);
    trigger.fields.reserved = ((pos >> sizeShift) & 1ull) ^ 1ull;  // lap 0 writes 1 (fifo_device.hpp:120)
    ProxyTrigger* slot = &triggers[pos & sizeMask];
    st_relaxed_sys(&slot->fst, trigger.fst);
    st_release_sys(&slot->snd, trigger.snd);  // commit word last: the payload is visible with it
    return pos;
  }
#endif
};

}  // namespace mscclpp_amd
