// Semaphore device handles for gfx950 (include/mscclpp/semaphore_device.hpp:17-135).
//
// Same pointer fields and member functions as the reference -- poll / wait / relaxedWait / signal /
// relaxedSignal / loadExpectedInbound / incExpectedInbound / loadInbound / loadInboundRelaxed --
// plus two fields of this library: `budget` (wall-clock bound of every wait, 10 ns ticks) and `err`
// (device error word that a timed-out wait records kErrSemaphoreTimeout in; may be null).  The host
// objects (semaphore.hpp) fill both.  HIP atomics here carry their scope explicitly: the expected
// counter is agent scope (this device only), tokens are system scope (written by a peer GPU or by a
// host proxy); `signal` is a system-scope release add into the peer's token
// (semaphore_device.hpp:84-90).
#pragma once

#include "device.hpp"

namespace mscclpp_amd {

namespace detail {
__device__ __forceinline__ bool spinUntilAtLeast(uint64_t* token, uint64_t want, bool acquire, uint64_t budget,
                                                 uint32_t* err) {
  SpinGuard g(budget ? budget : kDefaultSpinTicks);
  uint64_t seen;
  while ((seen = ld_relaxed_sys(token)) < want) {
    if (g.expired()) {
      // detail: a channel-handle wait (marker), the token value waited for and the one seen (low 32
      // bits): seen == want - 1 means the peer's last signal never arrived
      report_error_detail(err, kErrSemaphoreTimeout, 0x5E000000u, (uint32_t)want, (uint32_t)seen);
      return false;
    }
  }
  if (acquire) acquire_sys();  // the invalidate completes before later loads
  return true;
}
}  // namespace detail

// Host2DeviceSemaphore (semaphore_device.hpp:17-58): a host proxy (on behalf of the peer) writes
// `inboundToken`; the device waits for it.
struct Host2DeviceSemaphoreDeviceHandle {
  uint64_t* inboundToken;          // device memory, written by the proxy (a copy into it)
  uint64_t* expectedInboundToken;  // device memory
  uint64_t budget;                 // wait bound (10 ns ticks; 0 = kDefaultSpinTicks)
  uint32_t* err;                   // device error word (may be null)

#if defined(__HIP__)
  __device__ __forceinline__ uint64_t loadExpectedInbound() {
    return __hip_atomic_load(expectedInboundToken, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __device__ __forceinline__ uint64_t incExpectedInbound() {
    return __hip_atomic_fetch_add(expectedInboundToken, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  }
  __device__ __forceinline__ uint64_t loadInbound() { return ld_acquire_sys(inboundToken); }
  __device__ __forceinline__ bool poll() {
    const bool signaled = loadInbound() > loadExpectedInbound();
    if (signaled) incExpectedInbound();
    return signaled;
  }
  __device__ __forceinline__ void wait(int64_t maxSpinCount = 100000000) {
    (void)maxSpinCount;
    detail::spinUntilAtLeast(inboundToken, incExpectedInbound(), true, budget, err);
  }
#endif
};

// MemoryDevice2DeviceSemaphore (semaphore_device.hpp:61-135): the peer GPU adds into
// `inboundToken` (our memory, uncached) through its mapping `remoteInboundToken` of ours.
struct MemoryDevice2DeviceSemaphoreDeviceHandle {
  uint64_t* inboundToken;          // local, added to by the peer
  uint64_t* remoteInboundToken;    // the peer's inboundToken as mapped here
  uint64_t* expectedInboundToken;  // local wait counter
  uint64_t budget;                 // wait bound (10 ns ticks; 0 = kDefaultSpinTicks)
  uint32_t* err;                   // device error word (may be null)

#if defined(__HIP__)
  __device__ __forceinline__ uint64_t loadExpectedInbound() {
    return __hip_atomic_load(expectedInboundToken, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __device__ __forceinline__ uint64_t incExpectedInbound() {
    return __hip_atomic_fetch_add(expectedInboundToken, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  }
  __device__ __forceinline__ uint64_t loadInbound() { return ld_acquire_sys(inboundToken); }
  __device__ __forceinline__ uint64_t loadInboundRelaxed() { return ld_relaxed_sys(inboundToken); }
  // prior memory operations complete before the peer sees the signal
  __device__ __forceinline__ void signal() { add_release_sys(remoteInboundToken, 1); }
  __device__ __forceinline__ void relaxedSignal() { add_relaxed_sys(remoteInboundToken, 1); }
  __device__ __forceinline__ bool poll() {
    const bool signaled = loadInbound() > loadExpectedInbound();
    if (signaled) incExpectedInbound();
    return signaled;
  }
  __device__ __forceinline__ void wait(int64_t maxSpinCount = 100000000) {
    (void)maxSpinCount;
    detail::spinUntilAtLeast(inboundToken, incExpectedInbound(), true, budget, err);
  }
  __device__ __forceinline__ void relaxedWait(int64_t maxSpinCount = 100000000) {
    (void)maxSpinCount;
    detail::spinUntilAtLeast(inboundToken, incExpectedInbound(), false, budget, err);
  }
#endif
};

}  // namespace mscclpp_amd
