// Host cost of one small AllReduce call from C++ (no Python in the loop): n forked ranks, 1 KiB fp16,
// `iters` calls issued back to back on one stream; the time around the issuing loop alone is the
// host cost per call (the device catches up afterwards).  Rows: ncclAllReduce (selector + algorithm
// collection + launch), mscclppAmdCommAllReduce with the algorithm named (no selector), and an
// empty kernel launch on the same stream (the HIP runtime's own floor).  Rank 0 prints one JSON line.
//
//   bench_host_overhead <nranks> [iters]
#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "mscclpp_amd/mscclpp_amd.h"
#include "mscclpp_amd/nccl.h"

#define HIP_OK(x)                                                                          \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::_Exit(3);                                                                       \
    }                                                                                      \
  } while (0)
#define NCCL_OK(x)                                                          \
  do {                                                                      \
    int r_ = (int)(x);                                                      \
    if (r_ != 0) {                                                          \
      std::fprintf(stderr, "%s:%d %s -> %d\n", __FILE__, __LINE__, #x, r_); \
      std::_Exit(4);                                                        \
    }                                                                       \
  } while (0)

__global__ void emptyKernel() {}
// the LL kernels' argument block: one rank view + geometry + rank count + spin budget
struct BigArgs {
  mscclppAmdRankView v;
  uint64_t geom[6];
  int n;
  uint64_t budget;
};
__global__ void emptyKernelBigArgs(BigArgs a) {
  if (a.n < 0) a.v.err[0] = 1;  // never true: keeps the argument live
}
template <int N>
struct Words {
  uint64_t w[N];
};
template <int N>
__global__ void emptyKernelWords(Words<N> a) {
  if (a.w[N - 1] == 1) a.w[0] = 0;  // never true
}

struct PerCall {
  double host, drain;  // us per call: issuing loop alone; issuing loop + the device catching up
};

template <typename F>
static PerCall perCall(F&& f, int iters, hipStream_t s) {
  for (int i = 0; i < 20; ++i) f();
  HIP_OK(hipStreamSynchronize(s));
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < iters; ++i) f();
  const auto t1 = std::chrono::steady_clock::now();
  HIP_OK(hipStreamSynchronize(s));
  const auto t2 = std::chrono::steady_clock::now();
  return {std::chrono::duration<double, std::micro>(t1 - t0).count() / iters,
          std::chrono::duration<double, std::micro>(t2 - t0).count() / iters};
}

static int worker(int rank, int n, ncclUniqueId id, int iters) {
  int ndev = 0;
  HIP_OK(hipGetDeviceCount(&ndev));
  HIP_OK(hipSetDevice(rank % ndev));
  ncclComm_t comm;
  NCCL_OK(ncclCommInitRank(&comm, n, id, rank));
  hipStream_t s;
  HIP_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const size_t count = 512;  // 1 KiB of fp16: the one-hop LL8 path
  void *in, *out;
  HIP_OK(hipMalloc(&in, count * 2));
  HIP_OK(hipMalloc(&out, count * 2));
  HIP_OK(hipMemset(in, 0, count * 2));
  const PerCall empty = perCall([&] { hipLaunchKernelGGL(emptyKernel, dim3(1), dim3(64), 0, s); }, iters, s);
  BigArgs big{};
  big.n = n;
  const PerCall emptyBig =
      perCall([&] { hipLaunchKernelGGL(emptyKernelBigArgs, dim3(1), dim3(64), 0, s, big); }, iters, s);
  Words<1> w1{};
  Words<8> w8{};
  Words<16> w16{};
  Words<32> w32{};
  const double a8 = perCall([&] { hipLaunchKernelGGL(emptyKernelWords<1>, dim3(1), dim3(64), 0, s, w1); }, iters, s).host;
  const double a64 = perCall([&] { hipLaunchKernelGGL(emptyKernelWords<8>, dim3(1), dim3(64), 0, s, w8); }, iters, s).host;
  const double a128 =
      perCall([&] { hipLaunchKernelGGL(emptyKernelWords<16>, dim3(1), dim3(64), 0, s, w16); }, iters, s).host;
  const double a256 =
      perCall([&] { hipLaunchKernelGGL(emptyKernelWords<32>, dim3(1), dim3(64), 0, s, w32); }, iters, s).host;
  NCCL_OK(mscclppAmdCommBarrier(comm));
  const PerCall nccl = perCall([&] { ncclAllReduce(in, out, count, ncclFloat16, ncclSum, comm, s); }, iters, s);
  NCCL_OK(mscclppAmdCommBarrier(comm));
  const PerCall named = perCall(
      [&] { mscclppAmdCommAllReduce(comm, in, out, count, ncclFloat16, ncclSum, MSCCLPP_AMD_ALGO_ALLPAIR, 0, 0, s); },
      iters, s);
  NCCL_OK(mscclppAmdCommBarrier(comm));
  uint32_t err = 0;
  NCCL_OK(mscclppAmdCommGetDeviceError(comm, &err, 0));
  if (rank == 0)
    std::printf("{\"ranks\": %d, \"bytes\": %zu, \"iters\": %d, \"empty_launch_us\": [%.2f, %.2f], "
                "\"empty_launch_%zuB_args_us\": [%.2f, %.2f], \"empty_launch_host_us_by_arg_bytes\": "
                "{\"8\": %.2f, \"64\": %.2f, \"128\": %.2f, \"256\": %.2f}, "
                "\"ncclAllReduce_us\": [%.2f, %.2f], \"named_allpair_us\": [%.2f, %.2f], \"device_error\": %u, "
                "\"note\": \"[host issuing loop, host loop + drain] per call\"}\n",
                n, count * 2, iters, empty.host, empty.drain, sizeof(BigArgs), emptyBig.host, emptyBig.drain, a8, a64, a128, a256, nccl.host,
                nccl.drain, named.host, named.drain, err);
  std::fflush(stdout);
  NCCL_OK(ncclCommDestroy(comm));
  return err ? 5 : 0;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s <nranks> [iters]\n", argv[0]);
    return 2;
  }
  const int n = std::atoi(argv[1]);
  const int iters = argc > 2 ? std::atoi(argv[2]) : 2000;
  ncclUniqueId id;
  NCCL_OK(ncclGetUniqueId(&id));  // the root listens in this (parent) process; no GPU touched here
  std::vector<pid_t> pids;
  for (int r = 0; r < n; ++r) {
    pid_t pid = fork();
    if (pid < 0) return 3;
    if (pid == 0) std::_Exit(worker(r, n, id, iters));
    pids.push_back(pid);
  }
  int bad = 0;
  for (pid_t pid : pids) {
    int st = 0;
    waitpid(pid, &st, 0);
    if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) bad++;
  }
  return bad ? 1 : 0;
}
