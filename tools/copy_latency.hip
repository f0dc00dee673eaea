// Latency of the operations a PortChannel trigger turns into, one process, one GPU:
// submit -> complete of a 1 MiB device-to-device hipMemcpyAsync (default and NoCU), an 8-byte
// host-to-device hipMemcpyAsync, hipStreamWriteValue64 and a 1 MiB copy kernel, each on a
// non-blocking stream, first with the GPU otherwise idle, then while a one-wave kernel spins on
// another stream of the process (the state of a PortChannel kernel waiting for its peer).
// Prints one JSON line.  Build: hipcc --offload-arch=gfx950 -O2 tools/copy_latency.hip -o tools/bin/copy_latency
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <string>
#include <vector>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));   \
      std::exit(1);                                                                            \
    }                                                                                          \
  } while (0)

__global__ void copyKernel(uint4* d, const uint4* s, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) d[i] = s[i];
}

// spins until *stop != 0 or about 10 s of wall clock pass
__global__ void spinKernel(volatile int* stop) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (*stop == 0 && __builtin_amdgcn_s_memrealtime() - t0 < 1000000000ull) __builtin_amdgcn_s_sleep(2);
}

static double nowUs() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Stat {
  double med, min, max;
};
static Stat stat(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return {v[v.size() / 2], v.front(), v.back()};
}

int main() {
  const size_t bytes = 1 << 20;
  const int reps = 200;
  void *a, *b, *ua, *ub;
  uint64_t* tok;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  // uncached (fine-grained) buffers: what GpuBuffer allocates on AMD and what PortChannels copy between
  CK(hipExtMallocWithFlags(&ua, bytes, hipDeviceMallocUncached));
  CK(hipExtMallocWithFlags(&ub, bytes, hipDeviceMallocUncached));
  CK(hipExtMallocWithFlags((void**)&tok, 64, hipDeviceMallocUncached));
  uint64_t* slot;
  CK(hipHostMalloc((void**)&slot, 64, hipHostMallocDefault));
  int* stop;
  CK(hipHostMalloc((void**)&stop, 64, hipHostMallocMapped | hipHostMallocCoherent));
  int* dstop;
  CK(hipHostGetDevicePointer((void**)&dstop, stop, 0));
  hipStream_t cs, ks;
  CK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&ks, hipStreamNonBlocking));
  auto timeOp = [&](const char* name, auto&& op) {
    for (int i = 0; i < 5; ++i) op(i);  // warm
    CK(hipStreamSynchronize(cs));
    std::vector<double> wall, sub;
    for (int i = 0; i < reps; ++i) {
      const double t0 = nowUs();
      op(i);
      const double t1 = nowUs();
      CK(hipStreamSynchronize(cs));
      const double t2 = nowUs();
      sub.push_back(t1 - t0);
      wall.push_back(t2 - t0);
    }
    const Stat w = stat(wall), s = stat(sub);
    std::printf("\"%s\": {\"submit_to_done_us\": {\"median\": %.2f, \"min\": %.2f, \"max\": %.2f}, \"submit_us\": %.2f}",
                name, w.med, w.min, w.max, s.med);
  };
  auto all = [&](const char* tag) {
    std::printf("\"%s\": {", tag);
    timeOp("memcpy_d2d_1MiB", [&](int) { CK(hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, cs)); });
    std::printf(", ");
    timeOp("memcpy_d2d_nocu_1MiB", [&](int) { CK(hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDeviceNoCU, cs)); });
    std::printf(", ");
    timeOp("memcpy_h2d_8B", [&](int i) {
      slot[i % 8] = i;
      CK(hipMemcpyAsync(tok, &slot[i % 8], 8, hipMemcpyHostToDevice, cs));
    });
    std::printf(", ");
    timeOp("write_value64", [&](int i) { CK(hipStreamWriteValue64(cs, tok, (uint64_t)i, 0)); });
    std::printf(", ");
    timeOp("copy_kernel_1MiB", [&](int) {
      hipLaunchKernelGGL(copyKernel, dim3(256), dim3(256), 0, cs, (uint4*)b, (const uint4*)a, bytes / 16);
      CK(hipGetLastError());
    });
    std::printf(", ");
    timeOp("memcpy_d2d_plus_h2d_token", [&](int i) {
      CK(hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, cs));
      slot[i % 8] = i;
      CK(hipMemcpyAsync(tok, &slot[i % 8], 8, hipMemcpyHostToDevice, cs));
    });
    std::printf(", ");
    timeOp("memcpy_d2d_plus_write_value", [&](int i) {
      CK(hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, cs));
      CK(hipStreamWriteValue64(cs, tok, (uint64_t)i, 0));
    });
    std::printf(", ");
    timeOp("uncached_memcpy_d2d_1MiB", [&](int) { CK(hipMemcpyAsync(ub, ua, bytes, hipMemcpyDeviceToDevice, cs)); });
    std::printf(", ");
    timeOp("uncached_memcpy_d2d_nocu_1MiB",
           [&](int) { CK(hipMemcpyAsync(ub, ua, bytes, hipMemcpyDeviceToDeviceNoCU, cs)); });
    std::printf(", ");
    timeOp("uncached_copy_kernel_1MiB_256wg", [&](int) {
      hipLaunchKernelGGL(copyKernel, dim3(256), dim3(256), 0, cs, (uint4*)ub, (const uint4*)ua, bytes / 16);
      CK(hipGetLastError());
    });
    std::printf(", ");
    timeOp("uncached_copy_kernel_1MiB_1024wg", [&](int) {
      hipLaunchKernelGGL(copyKernel, dim3(1024), dim3(64), 0, cs, (uint4*)ub, (const uint4*)ua, bytes / 16);
      CK(hipGetLastError());
    });
    std::printf(", ");
    timeOp("cached_src_uncached_dst_memcpy_1MiB",
           [&](int) { CK(hipMemcpyAsync(ub, a, bytes, hipMemcpyDeviceToDevice, cs)); });
    std::printf(", ");
    timeOp("uncached_src_cached_dst_memcpy_1MiB",
           [&](int) { CK(hipMemcpyAsync(b, ua, bytes, hipMemcpyDeviceToDevice, cs)); });
    std::printf("}");
  };
  std::printf("{");
  all("idle");
  std::printf(", ");
  *stop = 0;
  hipLaunchKernelGGL(spinKernel, dim3(1), dim3(64), 0, ks, dstop);
  CK(hipGetLastError());
  all("beside_spinning_kernel");
  *stop = 1;
  CK(hipStreamSynchronize(ks));
  std::printf("}\n");
  return 0;
}
