// Host cost of one eager ncclAllReduce call on this library (diagnosis, not a test): two forked
// ranks on the current GPU(s), N back-to-back calls of a small LL bucket and of a bulk bucket, the
// host time per call measured around the enqueue loop alone (before the stream is drained) and
// around enqueue + drain.  Prints one line per case.
//   bench_call_overhead [calls]
#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "mscclpp_amd/mscclpp_amd.h"
#include "mscclpp_amd/nccl.h"

#define OK(cmd)                                                              \
  do {                                                                       \
    if ((cmd) != 0) {                                                        \
      std::fprintf(stderr, "%s:%d failed: %s\n", __FILE__, __LINE__, #cmd);  \
      std::_Exit(1);                                                         \
    }                                                                        \
  } while (0)

__global__ void emptyKernel(int* p) {
  if (p && threadIdx.x == 1023) *p = 0;
}

static int worker(int rank, int n, ncclUniqueId id, int calls) {
  int ndev = 0;
  OK(hipGetDeviceCount(&ndev));
  OK(hipSetDevice(rank % ndev));
  ncclComm_t comm;
  OK(ncclCommInitRank(&comm, n, id, rank));
  hipStream_t s;
  OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  {  // the floor: an empty kernel of the LL shape, launched back to back
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(emptyKernel, dim3(8), dim3(256), 0, s, nullptr);
    OK(hipStreamSynchronize(s));
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < calls; ++i) hipLaunchKernelGGL(emptyKernel, dim3(8), dim3(256), 0, s, nullptr);
    const auto t1 = std::chrono::steady_clock::now();
    OK(hipStreamSynchronize(s));
    const auto t2 = std::chrono::steady_clock::now();
    std::printf("rank %d empty kernel: host enqueue %.2f us/call, enqueue+drain %.2f us/call\n", rank,
                std::chrono::duration<double, std::micro>(t1 - t0).count() / calls,
                std::chrono::duration<double, std::micro>(t2 - t0).count() / calls);
  }
  for (size_t bytes : {(size_t)1 << 10, (size_t)64 << 10, (size_t)4 << 20}) {
    void *x, *y;
    OK(hipMalloc(&x, bytes));
    OK(hipMalloc(&y, bytes));
    OK(hipMemset(x, 0, bytes));
    const size_t count = bytes / 2;
    for (int i = 0; i < 20; ++i) OK(ncclAllReduce(x, y, count, ncclFloat16, ncclSum, comm, s));
    OK(hipStreamSynchronize(s));
    // line the ranks up before timing
    OK(ncclAllReduce(x, y, 1, ncclFloat16, ncclSum, comm, s));
    OK(hipStreamSynchronize(s));
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < calls; ++i) OK(ncclAllReduce(x, y, count, ncclFloat16, ncclSum, comm, s));
    const auto t1 = std::chrono::steady_clock::now();
    OK(hipStreamSynchronize(s));
    const auto t2 = std::chrono::steady_clock::now();
    const double enq = std::chrono::duration<double, std::micro>(t1 - t0).count() / calls;
    const double all = std::chrono::duration<double, std::micro>(t2 - t0).count() / calls;
    std::printf("rank %d bytes %zu: host enqueue %.2f us/call, enqueue+drain %.2f us/call\n", rank, bytes, enq, all);
    if (bytes <= (64u << 10)) {  // the same call with the algorithm named: no selector, no tuned lookup
      const int algo = MSCCLPP_AMD_ALGO_ALLPAIR;
      OK(mscclppAmdCommAllReduce(comm, x, y, count, ncclFloat16, ncclSum, algo, 0, 0, s));
      OK(hipStreamSynchronize(s));
      const auto u0 = std::chrono::steady_clock::now();
      for (int i = 0; i < calls; ++i) OK(mscclppAmdCommAllReduce(comm, x, y, count, ncclFloat16, ncclSum, algo, 0, 0, s));
      const auto u1 = std::chrono::steady_clock::now();
      OK(hipStreamSynchronize(s));
      std::printf("rank %d bytes %zu explicit allpair: host enqueue %.2f us/call\n", rank, bytes,
                  std::chrono::duration<double, std::micro>(u1 - u0).count() / calls);
    }
    std::fflush(stdout);
    OK(hipFree(x));
    OK(hipFree(y));
  }
  OK(ncclCommDestroy(comm));
  return 0;
}

int main(int argc, char** argv) {
  const int calls = argc > 1 ? std::atoi(argv[1]) : 2000;
  const int n = 2;
  ncclUniqueId id;
  OK(ncclGetUniqueId(&id));
  std::vector<pid_t> pids;
  for (int r = 0; r < n; ++r) {
    const pid_t pid = fork();
    if (pid == 0) std::_Exit(worker(r, n, id, calls));
    pids.push_back(pid);
  }
  int bad = 0;
  for (pid_t p : pids) {
    int st = 0;
    waitpid(p, &st, 0);
    bad += !(WIFEXITED(st) && WEXITSTATUS(st) == 0);
  }
  return bad ? 1 : 0;
}
