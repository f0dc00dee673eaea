// Device-memory helpers with the reference's spellings (include/mscclpp/gpu_utils.hpp):
// zero-initialised device / mapped-host / uncached arrays owned by shared or unique pointers, typed
// copies, the device guard and GpuBuffer -- which on AMD is uncached memory (gpu_utils.hpp:375-376,
// gpu_utils.cc:139-147) so that other GPUs and the copy engines see one copy of what kernels poll.
#ifndef MSCCLPP_AMD_GPU_UTILS_HPP_
#define MSCCLPP_AMD_GPU_UTILS_HPP_

#include <hip/hip_runtime_api.h>

#include <cstring>
#include <memory>
#include <string>
#include <utility>

#include "mscclpp_amd/core.hpp"
#include "mscclpp_amd/mscclpp_amd.h"

namespace mscclpp_amd {

// a failed runtime call throws CudaError carrying the hipError_t (gpu_utils.hpp MSCCLPP_CUDATHROW)
inline void gpuCheck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw CudaError(std::string("Call to ") + what + " failed", static_cast<int>(e));
}

// MSCCLPP_CUDATHROW (gpu_utils.hpp / errors.hpp): throw on a failed runtime call.  The calls are
// HIP's here; the macro keeps the reference's name so its callers read the same.
#define MSCCLPP_CUDATHROW(cmd)                                                                        \
  do {                                                                                                \
    const hipError_t err_ = (cmd);                                                                    \
    if (err_ != hipSuccess) ::mscclpp_amd::gpuCheck(err_, #cmd);                                      \
  } while (0)

// Make `deviceId` current for the guard's lifetime (gpu_utils.hpp:53-62).
struct CudaDeviceGuard {
  explicit CudaDeviceGuard(int deviceId) : deviceId_(deviceId), origDeviceId_(-1) {
    if (deviceId_ >= 0) {
      gpuCheck(hipGetDevice(&origDeviceId_), "hipGetDevice");
      if (origDeviceId_ != deviceId_) gpuCheck(hipSetDevice(deviceId_), "hipSetDevice");
    }
  }
  ~CudaDeviceGuard() {
    if (deviceId_ >= 0 && origDeviceId_ >= 0 && origDeviceId_ != deviceId_) (void)hipSetDevice(origDeviceId_);
  }
  CudaDeviceGuard(const CudaDeviceGuard&) = delete;
  CudaDeviceGuard& operator=(const CudaDeviceGuard&) = delete;
  int deviceId_;
  int origDeviceId_;
};

// Relaxed stream-capture mode for the guard's lifetime (the reference's AvoidCudaGraphCaptureGuard,
// gpu_utils.hpp:30-38): a set-up call made while another thread captures a graph neither joins nor
// invalidates that capture.
struct AvoidCudaGraphCaptureGuard {
  AvoidCudaGraphCaptureGuard() : mode_(hipStreamCaptureModeRelaxed) {
    (void)hipThreadExchangeStreamCaptureMode(&mode_);
  }
  ~AvoidCudaGraphCaptureGuard() { (void)hipThreadExchangeStreamCaptureMode(&mode_); }
  AvoidCudaGraphCaptureGuard(const AvoidCudaGraphCaptureGuard&) = delete;
  AvoidCudaGraphCaptureGuard& operator=(const AvoidCudaGraphCaptureGuard&) = delete;
  hipStreamCaptureMode mode_;
};

namespace detail {
// Run op(stream) on a stream of its own and wait for it: the reference's gpuCalloc / gpuMemcpy /
// gpuMemset are synchronous (gpu_utils.cc:120-128, :262-283) -- the fill or copy has completed on the
// device when they return.  (A bare hipMemset of device memory is asynchronous to the host: a host
// barrier after it does not order it before a peer's kernel)
template <typename F>
void syncOnOwnStream(F&& op, const char* what) {
  AvoidCudaGraphCaptureGuard guard;
  hipStream_t s = nullptr;
  gpuCheck(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreateWithFlags");
  hipError_t e = op(s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipStreamDestroy(s);
  gpuCheck(e, what);
}

inline void* gpuCalloc(size_t bytes) {
  AvoidCudaGraphCaptureGuard guard;
  void* p = nullptr;
  gpuCheck(hipMalloc(&p, bytes), "hipMalloc");
  try {
    syncOnOwnStream([&](hipStream_t s) { return hipMemsetAsync(p, 0, bytes, s); }, "hipMemsetAsync");
  } catch (...) {
    (void)hipFree(p);
    throw;
  }
  return p;
}

template <typename T>
std::shared_ptr<T> gpuCallocShared(size_t nelems = 1) {
  return std::shared_ptr<T>(static_cast<T*>(gpuCalloc(nelems * sizeof(T))), [](T* q) { (void)hipFree(q); });
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

template <class T = void>
struct GpuDeleter {
  void operator()(void* p) { (void)hipFree(p); }
};
template <class T = void>
struct GpuHostDeleter {
  void operator()(void* p) { (void)hipHostFree(p); }
};
template <class T = void>
struct GpuUncachedDeleter {
  void operator()(void* p) { (void)mscclppAmdFree(p); }
};
template <class T>
using UniqueGpuPtr = std::unique_ptr<T, GpuDeleter<T>>;
template <class T>
using UniqueGpuHostPtr = std::unique_ptr<T, GpuHostDeleter<T>>;
template <class T>
using UniqueGpuUncachedPtr = std::unique_ptr<T, GpuUncachedDeleter<T>>;

template <class T>
UniqueGpuPtr<T> gpuCallocUnique(size_t nelems = 1) {
  return UniqueGpuPtr<T>(static_cast<T*>(gpuCalloc(nelems * sizeof(T))));
}
// Zeroed host memory the GPU can reach (hipHostMalloc; mapped by default, gpu_utils.hpp:233-241).
inline void* gpuCallocHost(size_t bytes, unsigned int flags) {
  void* p = nullptr;
  gpuCheck(hipHostMalloc(&p, bytes, flags), "hipHostMalloc");
  std::memset(p, 0, bytes);
  return p;
}
template <class T>
std::shared_ptr<T> gpuCallocHostShared(size_t nelems = 1, unsigned int flags = hipHostMallocMapped) {
  return std::shared_ptr<T>(static_cast<T*>(gpuCallocHost(nelems * sizeof(T), flags)), GpuHostDeleter<T>());
}
template <class T>
UniqueGpuHostPtr<T> gpuCallocHostUnique(size_t nelems = 1, unsigned int flags = hipHostMallocMapped) {
  return UniqueGpuHostPtr<T>(static_cast<T*>(gpuCallocHost(nelems * sizeof(T), flags)));
}
template <class T>
UniqueGpuUncachedPtr<T> gpuCallocUncachedUnique(size_t nelems = 1) {
  void* p = nullptr;
  if (mscclppAmdMallocUncached(&p, nelems * sizeof(T)) != 0)
    throw Error("mscclppAmdMallocUncached failed", ErrorCode::SystemError);
  return UniqueGpuUncachedPtr<T>(static_cast<T*>(p));
}
}  // namespace detail

// Synchronous copy and fill, each on a stream of its own (gpu_utils.cc:262-283): complete on the
// device when they return, whatever the direction.
template <typename T = char>
void gpuMemcpy(T* dst, const T* src, size_t nelems, hipMemcpyKind kind = hipMemcpyDefault) {
  detail::syncOnOwnStream(
      [&](hipStream_t s) { return hipMemcpyAsync(dst, src, nelems * sizeof(T), kind, s); }, "hipMemcpyAsync");
}
template <typename T = char>
void gpuMemcpyAsync(T* dst, const T* src, size_t nelems, hipStream_t stream, hipMemcpyKind kind = hipMemcpyDefault) {
  AvoidCudaGraphCaptureGuard guard;
  gpuCheck(hipMemcpyAsync(dst, src, nelems * sizeof(T), kind, stream), "hipMemcpyAsync");
}
inline void gpuMemset(void* ptr, int value, size_t bytes) {
  detail::syncOnOwnStream([&](hipStream_t s) { return hipMemsetAsync(ptr, value, bytes, s); }, "hipMemsetAsync");
}

// No NVSwitch multicast or Hopper bulk copies on MI355X (gpu_utils.hpp:334-336).
inline bool isNvlsSupported() { return false; }
inline bool isBulkSupported() { return false; }

enum class GpuBufferGranularity { MultiCastMinimum, MultiCastRecommended };

// GpuBuffer (gpu_utils.hpp:350-405): `nelems` zeroed elements of uncached device memory on the current
// GPU -- the reference's AMD branch -- from this library's pool; the granularity only matters for
// NVLS multicast and is ignored.
template <class T = char>
class GpuBuffer {
 public:
  explicit GpuBuffer(size_t nelems, GpuBufferGranularity = GpuBufferGranularity::MultiCastMinimum)
      : nelems_(nelems), bytes_(nelems * sizeof(T)), deviceId_(-1) {
    if (nelems == 0) return;
    gpuCheck(hipGetDevice(&deviceId_), "hipGetDevice");
    memory_ = detail::gpuCallocUncachedShared<T>(nelems);
  }
  size_t nelems() const { return nelems_; }
  size_t bytes() const { return bytes_; }
  std::shared_ptr<T> memory() { return memory_; }
  T* data() { return memory_.get(); }
  int deviceId() const { return deviceId_; }

 private:
  size_t nelems_;
  size_t bytes_;
  int deviceId_;
  std::shared_ptr<T> memory_;
};

}  // namespace mscclpp_amd

#endif  // MSCCLPP_AMD_GPU_UTILS_HPP_
