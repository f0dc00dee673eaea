// Scoped atomics with the reference's spellings (include/mscclpp/atomic_device.hpp:43-65):
// atomicLoad / atomicStore / atomicFetchAdd<T, Scope>(ptr, [val,] memoryOrder) and the
// memoryOrder* / scope* constants.  The reference's HIP branch ignores its Scope argument and
// always emits system-scope __atomic_* (:49-65); here Scope is honoured on the device --
// scopeSystem for memory another GPU or the host touches, scopeDevice (agent: every XCD of this GPU)
// otherwise -- and host code gets the plain __atomic_* builtins.
#pragma once

#include <hip/hip_runtime.h>

namespace mscclpp_amd {

constexpr int memoryOrderRelaxed = __ATOMIC_RELAXED;
constexpr int memoryOrderAcquire = __ATOMIC_ACQUIRE;
constexpr int memoryOrderRelease = __ATOMIC_RELEASE;
constexpr int memoryOrderAcqRel = __ATOMIC_ACQ_REL;
constexpr int memoryOrderSeqCst = __ATOMIC_SEQ_CST;

constexpr int scopeSystem = __HIP_MEMORY_SCOPE_SYSTEM;
constexpr int scopeDevice = __HIP_MEMORY_SCOPE_AGENT;

template <typename T, int Scope = scopeSystem>
__host__ __device__ __forceinline__ T atomicLoad(const T* ptr, int memoryOrder) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __hip_atomic_load(const_cast<T*>(ptr), memoryOrder, Scope);
#else
  return __atomic_load_n(ptr, memoryOrder);
#endif
}

template <typename T, int Scope = scopeSystem>
__host__ __device__ __forceinline__ void atomicStore(T* ptr, const T& val, int memoryOrder) {
#if defined(__HIP_DEVICE_COMPILE__)
  __hip_atomic_store(ptr, val, memoryOrder, Scope);
#else
  __atomic_store_n(ptr, val, memoryOrder);
#endif
}

template <typename T, int Scope = scopeSystem>
__host__ __device__ __forceinline__ T atomicFetchAdd(T* ptr, const T& val, int memoryOrder) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __hip_atomic_fetch_add(ptr, val, memoryOrder, Scope);
#else
  return __atomic_fetch_add(ptr, val, memoryOrder);
#endif
}

}  // namespace mscclpp_amd
