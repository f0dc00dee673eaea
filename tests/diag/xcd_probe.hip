// Test diagnostics (not product code): read a buffer through EVERY XCD's L2 and count, per XCD, the
// words that differ from what the copy engine / host expects.  A word that only some XCDs see wrong
// is a stale line in those XCDs' L2s; a word every XCD sees wrong is missing from memory.
//   xcdCompare(buf, nwords, expect (host-pinned or device), out[8 * 4], stream)
//     out[x*4 + 0] = mismatching words seen by workgroups of XCD x (summed over its workgroups)
//     out[x*4 + 1] = first mismatching index (UINT64_MAX if none)
//     out[x*4 + 2] = last mismatching index
//     out[x*4 + 3] = workgroups that ran on XCD x
#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ __forceinline__ uint32_t xccId() {
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xF;
}

__global__ void __launch_bounds__(256) xcdCompareKernel(const uint32_t* buf, uint64_t n, const uint32_t* expect,
                                                        uint64_t* out) {
  const uint32_t x = xccId() & 7;
  uint64_t bad = 0, first = ~0ull, last = 0;
  for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const uint32_t g = buf[i];  // plain load: L1 -> this XCD's L2 -> memory
    const uint32_t e = __builtin_nontemporal_load(expect + i);
    if (g != e) {
      ++bad;
      first = i < first ? i : first;
      last = i > last ? i : last;
    }
  }
  if (bad) {
    atomicAdd((unsigned long long*)&out[x * 4 + 0], (unsigned long long)bad);
    atomicMin((unsigned long long*)&out[x * 4 + 1], (unsigned long long)first);
    atomicMax((unsigned long long*)&out[x * 4 + 2], (unsigned long long)last);
  }
  if (threadIdx.x == 0) atomicAdd((unsigned long long*)&out[x * 4 + 3], 1ull);
}

extern "C" int xcdCompare(const void* buf, uint64_t nwords, const void* expect, uint64_t* out, int workgroups,
                          hipStream_t s) {
  if (!buf || !expect || !out || workgroups <= 0 || workgroups > 4096) return 1;
  for (int x = 0; x < 8; ++x) {
    out[x * 4 + 0] = 0;
    out[x * 4 + 1] = ~0ull;
    out[x * 4 + 2] = 0;
    out[x * 4 + 3] = 0;
  }
  uint64_t* d = nullptr;
  if (hipMalloc(&d, 32 * sizeof(uint64_t)) != hipSuccess) return 2;
  hipError_t e = hipMemcpyAsync(d, out, 32 * sizeof(uint64_t), hipMemcpyHostToDevice, s);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(xcdCompareKernel, dim3(workgroups), dim3(256), 0, s, (const uint32_t*)buf, nwords,
                       (const uint32_t*)expect, d);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(out, d, 32 * sizeof(uint64_t), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipFree(d);
  return e == hipSuccess ? 0 : 3;
}
