// Host-proxy (PortChannel) device surface for gfx950: put / signal / flush / wait through the
// GPU -> host trigger FIFO (include/mscclpp/port_channel_device.hpp:12-195).
//
// BasePortChannelDeviceHandle { semaphoreId_, semaphore_, fifo_, flushDonePos_ } and
// PortChannelDeviceHandle { dst_, src_ } keep the reference's fields and member functions, so kernels
// written against include/mscclpp compile here after a namespace change.  Waits (wait, flush's wait
// for the proxy, a full FIFO) are bounded by the handles' wall-clock budgets and record their
// timeouts in the handles' error words.
#pragma once

#include "fifo_device.hpp"
#include "semaphore_device.hpp"

namespace mscclpp_amd {

using SemaphoreId = uint32_t;  // port_channel_device.hpp:14
using MemoryId = uint32_t;     // port_channel_device.hpp:18

namespace detail {
#if defined(__HIP__)
// Wait until the proxy has completed the TriggerSync pushed at `fifoPos`: it publishes
// flushDonePos = pos + 1 once the connection drained (port_channel_device.hpp:21-30).
__device__ __forceinline__ void waitFlush(uint64_t* flushDonePos, uint64_t fifoPos, uint64_t budget, uint32_t* err) {
  SpinGuard g(budget ? budget : kDefaultSpinTicks);
  while (ld_relaxed_sys(flushDonePos) <= fifoPos) {
    if (g.expired()) {
      report_error(err, kErrFifoTimeout);
      return;
    }
  }
  acquire_sys();
}
#endif
}  // namespace detail

struct BasePortChannelDeviceHandle {
  SemaphoreId semaphoreId_;
  Host2DeviceSemaphoreDeviceHandle semaphore_;
  FifoDeviceHandle fifo_;
  uint64_t* flushDonePos_;  // host-pinned, device-mapped: one past the last completed flush position

  BasePortChannelDeviceHandle() = default;
  __host__ __device__ BasePortChannelDeviceHandle(SemaphoreId semaphoreId, Host2DeviceSemaphoreDeviceHandle semaphore,
                                                  FifoDeviceHandle fifo, uint64_t* flushDonePos)
      : semaphoreId_(semaphoreId), semaphore_(semaphore), fifo_(fifo), flushDonePos_(flushDonePos) {}

#if defined(__HIP__)
  // A trigger carries 32-bit offsets and size (fifo_device.hpp:71-77; the reference asserts this in
  // debug builds and truncates in release ones).  A put that does not fit is not pushed at all --
  // no truncated copy, no signal for data that was not sent -- and kErrBadGeometry is recorded in
  // the FIFO's error word; larger transfers are split by the caller, as with the reference.
  __device__ __forceinline__ bool triggerFits(uint64_t dstOffset, uint64_t srcOffset, uint64_t size) {
    if (((dstOffset | srcOffset | size) >> TriggerBitsOffset) == 0) return true;
    report_error(fifo_.err, kErrBadGeometry);
    return false;
  }
  __device__ __forceinline__ void put(MemoryId dstId, uint64_t dstOffset, MemoryId srcId, uint64_t srcOffset,
                                     uint64_t size) {
    if (!triggerFits(dstOffset, srcOffset, size)) return;
    fifo_.push(ProxyTrigger(TriggerData, dstId, dstOffset, srcId, srcOffset, size, semaphoreId_));
  }
  __device__ __forceinline__ void put(MemoryId dstId, MemoryId srcId, uint64_t offset, uint64_t size) {
    put(dstId, offset, srcId, offset, size);
  }
  __device__ __forceinline__ void signal() { fifo_.push(ProxyTrigger(TriggerFlag, 0, 0, 0, 0, 0, semaphoreId_)); }
  __device__ __forceinline__ void putWithSignal(MemoryId dstId, uint64_t dstOffset, MemoryId srcId, uint64_t srcOffset,
                                               uint64_t size) {
    if (!triggerFits(dstOffset, srcOffset, size)) return;
    fifo_.push(ProxyTrigger(TriggerData | TriggerFlag, dstId, dstOffset, srcId, srcOffset, size, semaphoreId_));
  }
  __device__ __forceinline__ void putWithSignal(MemoryId dstId, MemoryId srcId, uint64_t offset, uint64_t size) {
    putWithSignal(dstId, offset, srcId, offset, size);
  }
  __device__ __forceinline__ void putWithSignalAndFlush(MemoryId dstId, uint64_t dstOffset, MemoryId srcId,
                                                       uint64_t srcOffset, uint64_t size,
                                                       int64_t maxSpinCount = 1000000) {
    (void)maxSpinCount;
    if (!triggerFits(dstOffset, srcOffset, size)) return;
    const uint64_t pos = fifo_.push(
        ProxyTrigger(TriggerData | TriggerFlag | TriggerSync, dstId, dstOffset, srcId, srcOffset, size, semaphoreId_));
    detail::waitFlush(flushDonePos_, pos, fifo_.budget, fifo_.err);
  }
  __device__ __forceinline__ void putWithSignalAndFlush(MemoryId dstId, MemoryId srcId, uint64_t offset, uint64_t size,
                                                       int64_t maxSpinCount = 1000000) {
    putWithSignalAndFlush(dstId, offset, srcId, offset, size, maxSpinCount);
  }
  __device__ __forceinline__ void flush(int64_t maxSpinCount = 1000000) {
    (void)maxSpinCount;
    const uint64_t pos = fifo_.push(ProxyTrigger(TriggerSync, 0, 0, 0, 0, 0, semaphoreId_));
    detail::waitFlush(flushDonePos_, pos, fifo_.budget, fifo_.err);
  }
  __device__ __forceinline__ bool poll() { return semaphore_.poll(); }
  __device__ __forceinline__ void wait(int64_t maxSpinCount = 10000000) { semaphore_.wait(maxSpinCount); }
#endif
};

struct PortChannelDeviceHandle : public BasePortChannelDeviceHandle {
  MemoryId dst_;
  MemoryId src_;

  PortChannelDeviceHandle() = default;
  __host__ __device__ PortChannelDeviceHandle(SemaphoreId semaphoreId, Host2DeviceSemaphoreDeviceHandle semaphore,
                                              FifoDeviceHandle fifo, MemoryId dst, MemoryId src, uint64_t* flushDonePos)
      : BasePortChannelDeviceHandle(semaphoreId, semaphore, fifo, flushDonePos), dst_(dst), src_(src) {}

#if defined(__HIP__)
  __device__ __forceinline__ void put(uint64_t dstOffset, uint64_t srcOffset, uint64_t size) {
    BasePortChannelDeviceHandle::put(dst_, dstOffset, src_, srcOffset, size);
  }
  __device__ __forceinline__ void put(uint64_t offset, uint64_t size) { put(offset, offset, size); }
  __device__ __forceinline__ void putWithSignal(uint64_t dstOffset, uint64_t srcOffset, uint64_t size) {
    BasePortChannelDeviceHandle::putWithSignal(dst_, dstOffset, src_, srcOffset, size);
  }
  __device__ __forceinline__ void putWithSignal(uint64_t offset, uint64_t size) {
    putWithSignal(offset, offset, size);
  }
  __device__ __forceinline__ void putWithSignalAndFlush(uint64_t dstOffset, uint64_t srcOffset, uint64_t size,
                                                       int64_t maxSpinCount = 1000000) {
    BasePortChannelDeviceHandle::putWithSignalAndFlush(dst_, dstOffset, src_, srcOffset, size, maxSpinCount);
  }
  __device__ __forceinline__ void putWithSignalAndFlush(uint64_t offset, uint64_t size) {
    putWithSignalAndFlush(offset, offset, size);
  }
#endif
};

}  // namespace mscclpp_amd
