// Small device-memory helpers with the reference's spellings (include/mscclpp/gpu_utils.hpp):
// zero-initialised device arrays owned by a shared_ptr, typed copies, and uncached allocation
// (hipExtMallocWithFlags(hipDeviceMallocUncached), gpu_utils.cc:139-147) for memory that other
// GPUs poll.
#ifndef MSCCLPP_AMD_GPU_UTILS_HPP_
#define MSCCLPP_AMD_GPU_UTILS_HPP_

#include <hip/hip_runtime_api.h>

#include <memory>
#include <string>

#include "mscclpp_amd/core.hpp"
#include "mscclpp_amd/mscclpp_amd.h"

namespace mscclpp_amd {

inline void gpuCheck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw Error(std::string(what) + ": " + hipGetErrorString(e), ErrorCode::SystemError);
}

namespace detail {
template <typename T>
std::shared_ptr<T> gpuCallocShared(size_t nelems = 1) {
  void* p = nullptr;
  gpuCheck(hipMalloc(&p, nelems * sizeof(T)), "hipMalloc");
  gpuCheck(hipMemset(p, 0, nelems * sizeof(T)), "hipMemset");
  return std::shared_ptr<T>(static_cast<T*>(p), [](T* q) { (void)hipFree(q); });
}
// Uncached memory comes from the library's process-lifetime pool (mscclppAmdMallocUncached, zeroed;
// released back to the pool, never to HIP, while the process runs: DESIGN.md §21).
template <typename T>
std::shared_ptr<T> gpuCallocUncachedShared(size_t nelems = 1) {
  void* p = nullptr;
  if (mscclppAmdMallocUncached(&p, nelems * sizeof(T)) != 0)
    throw Error("mscclppAmdMallocUncached failed", ErrorCode::SystemError);
  return std::shared_ptr<T>(static_cast<T*>(p), [](T* q) { (void)mscclppAmdFree(q); });
}
}  // namespace detail

template <typename T>
void gpuMemcpy(T* dst, const T* src, size_t nelems, hipMemcpyKind kind = hipMemcpyDefault) {
  gpuCheck(hipMemcpy(dst, src, nelems * sizeof(T), kind), "hipMemcpy");
}

}  // namespace mscclpp_amd

#endif  // MSCCLPP_AMD_GPU_UTILS_HPP_
