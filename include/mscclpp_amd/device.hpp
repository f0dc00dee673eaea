// mscclpp_amd device core: gfx950 memory operations with explicit cache scope, bounded spins and
// the device-side error word.  HIP for CDNA4 (gfx950) only.
//
// Replaces the reference's include/mscclpp/device.hpp, atomic_device.hpp:43-65 and
// poll_device.hpp:12-18 (POLL_MAYBE_JAILBREAK).  Differences by design:
//  * every scope is explicit.  The reference's HIP atomics ignore their scope argument and become
//    system-scope __atomic_* (atomic_device.hpp:49-65); here the scope is part of each call.
//  * 16-byte accesses use buffer instructions with cache-policy bits (sc0 sc1 = system,
//    sc1 = agent, nt = streaming) so a whole LL16 packet moves in one dwordx4.
//  * every spin is bounded by wall-clock time (s_memrealtime, 100 MHz) in every build, and a
//    timeout records a code in a device error word instead of hanging the GPU.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mscclpp_amd {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// Cache-policy bits of gfx950 buffer instructions (aux operand): sc0 = 1, nt = 2, sc1 = 16.
enum CachePolicy : int {
  kPlain = 0,
  kNonTemporal = 2,   // streaming: keep out of the way of reused lines
  kAgent = 16,        // sc1: bypass the CU's L1, coherent across the XCDs of one GPU
  kSystem = 17,       // sc0 sc1: write-through / read-through to memory, coherent across GPUs
};

// Error codes written to the device error word (first writer wins).
enum DeviceError : uint32_t {
  kErrNone = 0,
  kErrPacketTimeout = 1,     // an LL packet flag never arrived
  kErrSemaphoreTimeout = 2,  // a semaphore wait never completed
  kErrFifoTimeout = 3,       // a FIFO push found the ring full for too long
  kErrBadGeometry = 4,       // host passed inconsistent sizes
  kErrProxyFailure = 5,      // a host proxy's copy or token update failed (set from the host)
};

// Buffer resource over a raw pointer.  num_records = 0xFFFFFFFF: the whole 32-bit offset space is
// addressable; callers rebase the pointer for regions beyond 4 GiB.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0xFFFFFFFF, 0x00020000);
}

// A lane's strided walk over n units of Unit bytes (i = tid, tid + nthreads, ...) through buffer
// resources, whose offsets are 32 bits: f(i, w0, off) with off = (i - w0) * Unit, the byte offset
// of unit i from unit w0, where the caller's resources start.  Up to 4 GiB (every bucket in
// practice) w0 is 0 throughout and the caller's resources are loop-invariant; beyond, the walk goes
// window by window of 2 GiB with w0 the window's first unit (uniform across the wave), so a buffer
// of any size is addressed exactly as the reference's 64-bit pointer arithmetic addresses it.
template <uint32_t Unit, typename F>
__host__ __device__ __forceinline__ void for_each_strided(uint64_t n, uint64_t tid, uint64_t nthreads, F&& f) {
  if (n * Unit <= 0xFFFFFFFFull) {
    for (uint64_t i = tid; i < n; i += nthreads) f(i, (uint64_t)0, (uint32_t)(i * Unit));
    return;
  }
  constexpr uint64_t kWindowUnits = (1ull << 31) / Unit;
  for (uint64_t w0 = 0; w0 < n; w0 += kWindowUnits) {
    const uint64_t w1 = n - w0 < kWindowUnits ? n : w0 + kWindowUnits;
    uint64_t i = tid >= w0 ? tid : tid + (w0 - tid + nthreads - 1) / nthreads * nthreads;
    for (; i < w1; i += nthreads) f(i, w0, (uint32_t)((i - w0) * Unit));
  }
}

template <int Policy>
__device__ __forceinline__ u32x4 load16(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, Policy);
}
template <int Policy>
__device__ __forceinline__ void store16(__amdgpu_buffer_rsrc_t r, uint32_t byte_off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, byte_off, 0, Policy);
}
template <int Policy>
__device__ __forceinline__ u32x2 load8(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  return __builtin_amdgcn_raw_buffer_load_b64(r, byte_off, 0, Policy);
}
template <int Policy>
__device__ __forceinline__ void store8(__amdgpu_buffer_rsrc_t r, uint32_t byte_off, u32x2 v) {
  __builtin_amdgcn_raw_buffer_store_b64(v, r, byte_off, 0, Policy);
}
template <int Policy>
__device__ __forceinline__ uint32_t load4(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, Policy);
}
template <int Policy>
__device__ __forceinline__ void store4(__amdgpu_buffer_rsrc_t r, uint32_t byte_off, uint32_t v) {
  __builtin_amdgcn_raw_buffer_store_b32(v, r, byte_off, 0, Policy);
}

// Wall clock in 10 ns ticks (s_memrealtime runs at a constant 100 MHz on gfx950).
__device__ __forceinline__ uint64_t wall_ticks() { return __builtin_amdgcn_s_memrealtime(); }

// Bounded spin bookkeeping.  `budget_ticks` == 0 means "never time out" (not used by the library;
// every library call passes a finite budget).
struct SpinGuard {
  uint64_t deadline;
  uint32_t iter;
  __device__ __forceinline__ explicit SpinGuard(uint64_t budget_ticks)
      : deadline(budget_ticks ? wall_ticks() + budget_ticks : ~0ull), iter(0) {}
  // Returns true when the caller must give up.  Reads the clock once every 256 polls.
  __device__ __forceinline__ bool expired() {
    if ((++iter & 255u) != 0) return false;
    return wall_ticks() > deadline;
  }
};

// Spin budget of the reference-spelled waits that carry no budget of their own (LL16Packet::read,
// copyFromPackets, ...): 20 s of wall clock, the library default (MSCCLPP_AMD_SPIN_TIMEOUT_MS).
//
// The reference's `maxSpinCount` arguments (poll_device.hpp:12-18) are accepted for source
// compatibility and, as in the reference's release build (MSCCLPP_ASSERT_DEVICE is active only with
// DEBUG_BUILD, assert_device.hpp), do not end a wait.  What ends a stuck wait here is the
// wall-clock budget, in every build: the wait returns and the error word (when the handle has one)
// records the timeout.
constexpr uint64_t kDefaultSpinTicks = 2000000000ull;

__device__ __forceinline__ void report_error(uint32_t* err, uint32_t code) {
  if (err) {
    uint32_t expected = kErrNone;
    __hip_atomic_compare_exchange_strong(err, &expected, code, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// As report_error; the first reporter also records three diagnostic words in err[1..3].  Every
// error word the library allocates or accepts is 4 words (16 bytes) or more: err[0] the code,
// err[1..3] the detail of the first error.
__device__ __forceinline__ void report_error_detail(uint32_t* err, uint32_t code, uint32_t a, uint32_t b, uint32_t c) {
  if (!err) return;
  uint32_t expected = kErrNone;
  if (__hip_atomic_compare_exchange_strong(err, &expected, code, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_SYSTEM)) {
    __hip_atomic_store(err + 1, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(err + 2, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(err + 3, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// A packet that never carried the expected flag: err[1] = the flag waited for, err[2] = where the
// packet sits (the byte offset of the packet, or of the 32-byte unit, from the polled region's
// base), err[3] = the flag word last read there (the first of the packet's flag words that differed).
// One failure then says which round (flag) and which packet stopped, and whether the slot held an
// older round's flag (the packet was never written, or was overwritten after it landed) or zero (the
// slot was cleared after the peer wrote it).
__device__ __forceinline__ void report_packet_timeout(uint32_t* err, uint32_t flag, uint64_t where, uint32_t seen) {
  report_error_detail(err, kErrPacketTimeout, flag, (uint32_t)where, seen);
}

// Release / acquire with the wait the fence needs on gfx950 (MI355X_MICROARCH.md, "Compiler hazard"
// and the acquire row of the fence table).  A release fence writes the XCD's L2 back
// (`buffer_wbl2`) and an acquire fence invalidates (`buffer_inv`); both complete asynchronously.
// With a release ATOMIC alone the compiler drops the wait after the write-back whenever the wave's
// vmcnt is provably empty (e.g. after a waited load of the peer's token address), and the signal
// then overtakes the write-back: here 8 in-process ranks lost the plain stores of two workgroups
// (mscclpp-test allreduce5), which the peers on the same XCD had already read.  So: fence, explicit
// `s_waitcnt vmcnt(0)`, then a RELAXED atomic -- and after an acquire fence the same wait, so the
// invalidate has completed before the workgroup barrier releases the other waves' loads.
__device__ __forceinline__ void release_sys() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void release_agent() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void acquire_sys() {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void acquire_agent() {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Relaxed system-scope 64-bit load / store / add (global_* sc0 sc1), used for tokens and flags.
__device__ __forceinline__ uint64_t ld_relaxed_sys(const uint64_t* p) {
  return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// A load that later loads of this wave may depend on (one acquire per call: poll with
// ld_relaxed_sys in loops and acquire once after them where the loop is hot).
__device__ __forceinline__ uint64_t ld_acquire_sys(const uint64_t* p) {
  const uint64_t v = __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  acquire_sys();
  return v;
}
__device__ __forceinline__ void st_relaxed_sys(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_release_sys(uint64_t* p, uint64_t v) {
  release_sys();
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t add_release_sys(uint64_t* p, uint64_t v) {
  release_sys();
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t add_relaxed_sys(uint64_t* p, uint64_t v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t add_release_agent(uint64_t* p, uint64_t v) {
  release_agent();
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace mscclpp_amd
