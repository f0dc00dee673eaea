// Grid-level synchronization for kernels written against the reference's
// include/mscclpp/concurrency_device.hpp: DeviceSyncer (a grid barrier over the first `blockNum`
// workgroups, :28-69) and DeviceSemaphore (a device-wide counting semaphore, :97-132).  Both are
// plain zero-initialisable structs meant to live in `__device__` globals, as the reference's are.
//
// gfx950 details.  The barrier is a generation counter: the last workgroup to arrive subtracts the
// generation's arrivals from the count and then bumps the generation, the others poll the
// generation -- no shared "previous flag" that every workgroup rewrites.  A workgroup's stores are written back from its XCD's L2
// before it arrives (agent-scope release: the barrier spans the 8 XCDs) and the L2 is invalidated
// after it leaves (acquire), so what one workgroup stored before sync() is what every other one
// loads after it.  The waits poll with `s_sleep 1` between loads.  maxSpinCount bounds the polls
// (negative: unbounded); where the reference asserts when it runs out, this one leaves the wait and
// records it in timedOut(), since a device trap could take the whole GPU down.
#pragma once

#include "device.hpp"

namespace mscclpp_amd {

struct DeviceSyncer {
  DeviceSyncer() = default;

#if defined(__HIP__)
  // Every thread of the first `blockNum` workgroups calls this; it returns once all of them have.
  __device__ __forceinline__ void sync(int blockNum, int64_t maxSpinCount = 100000000) {
    __syncthreads();
    if (blockNum <= 1) return;
    if (threadIdx.x == 0) {
      const uint32_t g = __hip_atomic_load(&gen_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      release_agent();
      if (__hip_atomic_fetch_add(&count_, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)blockNum - 1) {
        // Take this generation's arrivals back out, and only then publish the new generation: a
        // waiter that sees it may enter the next sync() at once, and its arrival must not be
        // overwritten by a reset still in flight.  A subtraction (not a store of 0) keeps any such
        // arrival whatever the order, and the release (fence + s_waitcnt) completes it before the
        // generation store is issued.
        __hip_atomic_fetch_sub(&count_, (uint32_t)blockNum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        release_agent();
        __hip_atomic_store(&gen_, g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        int64_t spins = 0;
        while (__hip_atomic_load(&gen_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) {
          __builtin_amdgcn_s_sleep(1);
          if (maxSpinCount >= 0 && ++spins > maxSpinCount) {
            __hip_atomic_store(&timedOut_, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
        }
      }
      acquire_agent();
    }
    __syncthreads();
  }
  // A wait of this barrier ran out of spins (sticky).
  __device__ __forceinline__ bool timedOut() const {
    return __hip_atomic_load(const_cast<uint32_t*>(&timedOut_), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  }
#endif

 private:
  uint32_t count_ = 0;     // workgroups arrived in the current generation
  uint32_t gen_ = 0;       // generations completed
  uint32_t timedOut_ = 0;
};

struct DeviceSemaphore {
  DeviceSemaphore() = default;
  DeviceSemaphore(int initialValue) : semaphore_(initialValue) {}

#if defined(__HIP__)
  __device__ __forceinline__ void set(int value) {
    release_agent();
    __hip_atomic_store(&semaphore_, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // Take one unit; when none was left, wait until a release has handed one back.
  __device__ __forceinline__ void acquire(int maxSpinCount = -1) {
    const int old = __hip_atomic_fetch_add(&semaphore_, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old <= 0) {
      int64_t spins = 0;
      while (__hip_atomic_load(&semaphore_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < old) {
        __builtin_amdgcn_s_sleep(1);
        if (maxSpinCount >= 0 && ++spins > maxSpinCount) break;
      }
    }
    acquire_agent();
  }
  __device__ __forceinline__ void release() {
    release_agent();
    __hip_atomic_fetch_add(&semaphore_, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#endif

 private:
  int semaphore_ = 0;
};

}  // namespace mscclpp_amd
