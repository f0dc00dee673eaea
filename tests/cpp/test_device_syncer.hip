// DeviceSyncer back to back (include/mscclpp/concurrency_device.hpp:28-69, spelled as the reference's
// kernels spell it): a grid of co-resident workgroups calls sync() twice per round for many rounds.
// Round i: every workgroup stores i into its slot, sync(), every workgroup reads all slots and
// counts the ones that do not hold i, sync() again before the next round overwrites them.  A lost
// arrival (the reset of one generation wiping an early arrival of the next) would leave the grid
// waiting out the spin bound: timedOut() then reports it, and stale slots show as mismatches.
//
//   test_device_syncer gpu [blocks] [rounds]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>

#include <mscclpp/concurrency_device.hpp>

__device__ mscclpp::DeviceSyncer gSyncer;

__global__ void syncerRounds(volatile int* slots, int rounds, unsigned long long* mismatches, int* timedOut) {
  for (int i = 1; i <= rounds; ++i) {
    if (threadIdx.x == 0) slots[blockIdx.x] = i;
    gSyncer.sync(gridDim.x, 50000000);
    unsigned long long bad = 0;
    for (int b = threadIdx.x; b < (int)gridDim.x; b += blockDim.x) bad += slots[b] != i;
    if (bad) atomicAdd(mismatches, bad);
    gSyncer.sync(gridDim.x, 50000000);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *timedOut = gSyncer.timedOut() ? 1 : 0;
}

#define HIP_OK(x)                                                            \
  do {                                                                       \
    hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) {                                                  \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                              \
    }                                                                        \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 2 || std::string(argv[1]) != "gpu") {
    std::fprintf(stderr, "usage: %s gpu [blocks] [rounds]\n", argv[0]);
    return 2;
  }
  const int blocks = argc > 2 ? std::atoi(argv[2]) : 128;
  const int rounds = argc > 3 ? std::atoi(argv[3]) : 20000;
  hipDeviceProp_t prop;
  HIP_OK(hipGetDeviceProperties(&prop, 0));
  if (blocks < 2 || blocks > prop.multiProcessorCount) {  // one 256-lane workgroup per CU: all co-resident
    std::fprintf(stderr, "blocks must be 2..%d\n", prop.multiProcessorCount);
    return 2;
  }
  int* slots = nullptr;
  int* timedOut = nullptr;
  unsigned long long* mism = nullptr;
  HIP_OK(hipMalloc((void**)&slots, blocks * sizeof(int)));
  HIP_OK(hipMemset(slots, 0, blocks * sizeof(int)));
  HIP_OK(hipMalloc((void**)&mism, sizeof(*mism)));
  HIP_OK(hipMemset(mism, 0, sizeof(*mism)));
  HIP_OK(hipMalloc((void**)&timedOut, sizeof(int)));
  HIP_OK(hipMemset(timedOut, 0, sizeof(int)));
  for (int launch = 0; launch < 3; ++launch) {  // the syncer's state carries over from launch to launch
    hipLaunchKernelGGL(syncerRounds, dim3(blocks), dim3(256), 0, 0, slots, rounds, mism, timedOut);
    HIP_OK(hipGetLastError());
    HIP_OK(hipDeviceSynchronize());
  }
  unsigned long long m = 0;
  int to = 0;
  HIP_OK(hipMemcpy(&m, mism, sizeof(m), hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(&to, timedOut, sizeof(to), hipMemcpyDeviceToHost));
  std::printf("blocks %d rounds %d x 3 launches: mismatches %llu timedOut %d\n", blocks, rounds, m, to);
  if (m || to) {
    std::printf("gpu FAILED\n");
    return 1;
  }
  std::printf("gpu OK\n");
  return 0;
}
