// A user-defined collective plugged into ncclAllGather through the C++ algorithm interface -- the API
// sequence of the reference's plugin example (examples/customized-collective-algorithm/): an
// AlgorithmBuilder whose NativeAlgorithm sets up PortChannels with the public host API (connect,
// registerMemory / sendMemory / recvMemory, ProxyService::buildAndAddSemaphore / addMemory /
// portChannel), a selector registered with collective::AlgorithmCollectionBuilder before
// ncclCommInitRank, one context per (input, output, sizes) key, then ncclAllGather calls -- direct and
// captured in a HIP graph -- that must reach the user's kernel.  The algorithm itself is this test's
// own: one workgroup per peer, whose lane 0 issues putWithSignalAndFlush and waits for the peer's
// signal.  Everything is included and spelled as against the reference (<mscclpp/...>, mscclpp::).
//
//   test_customized_allgather gpu <nranks> [floats per rank] [cached | uncached | refuse | direct]
//
// The PortChannel destination contract: `cached` (hipMalloc receive buffer) is
// exact -- the receiving kernel only waits for the signal, the data is read after it -- and
// ProxyService warns once that the destination is cached device memory; `uncached` allocates the
// receive buffer from the uncached pool (no warning); `refuse` runs with
// MSCCLPP_AMD_PORT_CHANNEL_DST=strict and expects the first ncclAllGather to return
// ncclInvalidUsage on every rank (ProxyService::addMemory refuses the peer's buffer before any
// semaphore is built, so no rank is left waiting for another); `direct` allocates the receive buffer
// with hipExtMallocWithFlags(hipDeviceMallocUncached) itself -- not from the pool -- and runs under
// strict: it is coherent, so it must be accepted, exact, with no warning.
#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <memory>
#include <mscclpp/algorithm.hpp>
#include <mscclpp/core.hpp>
#include <mscclpp/ext/collectives/algorithm_collection_builder.hpp>
#include <mscclpp/ext/nccl/nccl.h>
#include <mscclpp/gpu_utils.hpp>
#include <mscclpp/port_channel.hpp>
#include <string>
#include <vector>

#include "mscclpp_amd/mscclpp_amd.h"

namespace {

int gRank = -1;

void require(bool ok, const char* what, int line) {
  if (ok) return;
  std::fprintf(stderr, "[rank %d] line %d: %s\n", gRank, line, what);
  std::exit(1);
}
#define REQUIRE(x) require((x), #x, __LINE__)

using PortHandle = mscclpp::DeviceHandle<mscclpp::PortChannel>;

// Workgroup p serves peer channel p: my whole block goes to offset rank * bytes of the peer's output,
// flushed, and then the peer's block is awaited through the same channel's semaphore.
__global__ void gatherThroughPeers(PortHandle* channels, uint64_t dstOffset, uint64_t bytes) {
  if (threadIdx.x != 0) return;
  PortHandle ch = channels[blockIdx.x];
  ch.putWithSignalAndFlush(dstOffset, 0, bytes);
  ch.wait();
}

// What one (input, output, size) key needs at call time; the registered memories stay referenced
// for as long as the channels that point into them.
struct GatherPlan {
  int rank = 0;
  int nPeers = 0;
  std::shared_ptr<PortHandle> channels;
  std::vector<mscclpp::RegisteredMemory> pinned;
};

std::atomic<int> gSetups{0}, gPlans{0}, gLaunches{0};

// The per-communicator state behind the algorithm: connections to every peer and one proxy.
class PeerGather {
 public:
  ~PeerGather() {
    if (proxy_) proxy_->stopProxy();
  }

  void setUp(std::shared_ptr<mscclpp::Communicator> comm) {
    ++gSetups;
    const int me = comm->bootstrap()->getRank(), n = comm->bootstrap()->getNranks();
    std::map<int, std::shared_future<mscclpp::Connection>> pending;
    for (int q = 0; q < n; ++q)
      if (q != me) pending.emplace(q, comm->connect(mscclpp::Transport::CudaIpc, q));
    for (auto& kv : pending) links_.push_back({kv.first, kv.second.get()});
    proxy_ = std::make_shared<mscclpp::ProxyService>();
    proxy_->startProxy();
  }

  std::shared_ptr<void> plan(std::shared_ptr<mscclpp::Communicator> comm, const void* in, void* out, size_t bytes) {
    ++gPlans;
    auto p = std::make_shared<GatherPlan>();
    p->rank = comm->bootstrap()->getRank();
    p->nPeers = (int)links_.size();
    const int n = p->nPeers + 1;
    auto src = comm->registerMemory(const_cast<void*>(in), bytes, mscclpp::Transport::CudaIpc);
    auto dst = comm->registerMemory(out, bytes * n, mscclpp::Transport::CudaIpc);
    std::vector<std::shared_future<mscclpp::RegisteredMemory>> theirs;
    for (const Link& l : links_) {
      comm->sendMemory(dst, l.peer, 0);
      theirs.push_back(comm->recvMemory(l.peer, 0));
    }
    const mscclpp::MemoryId srcId = proxy_->addMemory(src);
    std::vector<PortHandle> handles;
    for (size_t i = 0; i < links_.size(); ++i) {
      mscclpp::RegisteredMemory remote = theirs[i].get();
      const mscclpp::MemoryId dstId = proxy_->addMemory(remote);
      const mscclpp::SemaphoreId sem = proxy_->buildAndAddSemaphore(*comm, links_[i].conn);
      handles.push_back(mscclpp::deviceHandle(proxy_->portChannel(sem, dstId, srcId)));
      p->pinned.push_back(remote);
    }
    p->pinned.push_back(src);
    p->pinned.push_back(dst);
    p->channels = mscclpp::detail::gpuCallocShared<PortHandle>(handles.size());
    mscclpp::gpuMemcpy(p->channels.get(), handles.data(), handles.size(), hipMemcpyHostToDevice);
    return p;
  }

  mscclpp::CommResult launch(const std::shared_ptr<void>& ctx, size_t bytes, hipStream_t stream) {
    ++gLaunches;
    const auto* p = static_cast<const GatherPlan*>(ctx.get());
    hipLaunchKernelGGL(gatherThroughPeers, dim3(p->nPeers), dim3(64), 0, stream, p->channels.get(),
                       (uint64_t)p->rank * bytes, (uint64_t)bytes);
    return hipGetLastError() == hipSuccess ? mscclpp::CommResult::CommSuccess
                                           : mscclpp::CommResult::CommInternalError;
  }

 private:
  struct Link {
    int peer;
    mscclpp::Connection conn;
  };
  std::vector<Link> links_;
  std::shared_ptr<mscclpp::ProxyService> proxy_;
};

class PeerGatherBuilder : public mscclpp::AlgorithmBuilder {
 public:
  std::shared_ptr<mscclpp::Algorithm> build() override {
    auto state = std::make_shared<PeerGather>();
    return std::make_shared<mscclpp::NativeAlgorithm>(
        "peer_gather", "allgather",
        [state](std::shared_ptr<mscclpp::Communicator> comm) { state->setUp(comm); },
        [state](const std::shared_ptr<void> ctx, const void*, void*, size_t inBytes, size_t, mscclpp::DataType,
                mscclpp::ReduceOp, hipStream_t stream, int, int, const std::unordered_map<std::string, uintptr_t>&,
                mscclpp::DataType) { return state->launch(ctx, inBytes, stream); },
        [state](std::shared_ptr<mscclpp::Communicator> comm, const void* in, void* out, size_t inBytes, size_t,
                mscclpp::DataType) { return state->plan(comm, in, out, inBytes); },
        [](const void* in, void* out, size_t inBytes, size_t outBytes, mscclpp::DataType, bool) {
          return mscclpp::AlgorithmCtxKey{const_cast<void*>(in), out, inBytes, outBytes, 0};
        });
  }
};

float expectedValue(int r, size_t i) { return (float)(r * 7919 + (int)(i % 65521)) * 0.5f; }

int runRank(int rank, int n, ncclUniqueId id, size_t count, const std::string& mode) {
  gRank = rank;
  int ndev = 0;
  REQUIRE(hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0);
  REQUIRE(hipSetDevice(rank % ndev) == hipSuccess);
  // the plugin and its selector go in before the communicator exists
  auto registry = mscclpp::collective::AlgorithmCollectionBuilder::getInstance();
  registry->addAlgorithmBuilder(std::make_shared<PeerGatherBuilder>());
  registry->setAlgorithmSelector(
      [](const std::unordered_map<std::string, std::unordered_map<std::string, std::shared_ptr<mscclpp::Algorithm>>>&
             byCollective,
         const mscclpp::CollectiveRequest& req) -> std::shared_ptr<mscclpp::Algorithm> {
        auto c = byCollective.find(req.collective);
        if (c == byCollective.end()) return nullptr;
        auto a = c->second.find("peer_gather");
        return a == c->second.end() ? nullptr : a->second;
      });
  const size_t bytes = count * sizeof(float);
  float* send = nullptr;
  float* recv = nullptr;
  REQUIRE(hipMalloc(&send, bytes) == hipSuccess);
  if (mode == "uncached")
    REQUIRE(mscclppAmdMallocUncached((void**)&recv, bytes * n) == 0);
  else if (mode == "direct")
    REQUIRE(hipExtMallocWithFlags((void**)&recv, bytes * n, hipDeviceMallocUncached) == hipSuccess);
  else
    REQUIRE(hipMalloc(&recv, bytes * n) == hipSuccess);
  if (mode == "refuse" || mode == "direct") setenv("MSCCLPP_AMD_PORT_CHANNEL_DST", "strict", 1);
  std::vector<float> mine(count);
  for (size_t i = 0; i < count; ++i) mine[i] = expectedValue(rank, i);
  REQUIRE(hipMemcpy(send, mine.data(), bytes, hipMemcpyHostToDevice) == hipSuccess);
  // AllGather's own block: the algorithm only moves the peers' blocks
  auto resetOutput = [&] {
    REQUIRE(hipMemset(recv, 0xFF, bytes * n) == hipSuccess);
    REQUIRE(hipMemcpy(recv + rank * count, send, bytes, hipMemcpyDeviceToDevice) == hipSuccess);
    // both fills have landed before the barrier that lets the peers write into `recv` (DESIGN.md §8:
    // a host barrier orders host calls, not device work still queued)
    REQUIRE(hipDeviceSynchronize() == hipSuccess);
  };
  resetOutput();
  hipStream_t stream;
  REQUIRE(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) == hipSuccess);
  ncclComm_t comm;
  REQUIRE(ncclCommInitRank(&comm, n, id, rank) == ncclSuccess);
  auto verify = [&](const char* stage) {
    std::vector<float> all(count * n);
    REQUIRE(hipMemcpy(all.data(), recv, bytes * n, hipMemcpyDeviceToHost) == hipSuccess);
    size_t wrong = 0;
    for (int r = 0; r < n; ++r)
      for (size_t i = 0; i < count; ++i) wrong += all[r * count + i] != expectedValue(r, i);
    if (wrong) std::fprintf(stderr, "[rank %d] %s: %zu of %zu floats wrong\n", rank, stage, wrong, count * n);
    REQUIRE(wrong == 0);
  };
  if (mode == "refuse") {
    REQUIRE(ncclAllGather(send, recv, count, ncclFloat, comm, stream) == ncclInvalidUsage);
    REQUIRE(std::string(ncclGetLastError(comm)).find("cached device memory") != std::string::npos);
  } else {
    REQUIRE(ncclAllGather(send, recv, count, ncclFloat, comm, stream) == ncclSuccess);
    REQUIRE(hipStreamSynchronize(stream) == hipSuccess);
    verify("direct call");
    resetOutput();
    REQUIRE(mscclppAmdCommBarrier(comm) == 0);  // no peer still writes into the reset buffer
    constexpr int kCaptured = 8;
    hipGraph_t graph;
    hipGraphExec_t exec;
    REQUIRE(hipStreamBeginCapture(stream, hipStreamCaptureModeGlobal) == hipSuccess);
    for (int i = 0; i < kCaptured; ++i)
      REQUIRE(ncclAllGather(send, recv, count, ncclFloat, comm, stream) == ncclSuccess);
    REQUIRE(hipStreamEndCapture(stream, &graph) == hipSuccess);
    REQUIRE(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0) == hipSuccess);
    hipEvent_t t0, t1;
    REQUIRE(hipEventCreate(&t0) == hipSuccess && hipEventCreate(&t1) == hipSuccess);
    REQUIRE(hipEventRecord(t0, stream) == hipSuccess);
    REQUIRE(hipGraphLaunch(exec, stream) == hipSuccess);
    REQUIRE(hipEventRecord(t1, stream) == hipSuccess);
    REQUIRE(hipEventSynchronize(t1) == hipSuccess);
    float ms = 0;
    REQUIRE(hipEventElapsedTime(&ms, t0, t1) == hipSuccess);
    verify("graph replay");
    ncclResult_t async = ncclSuccess;
    REQUIRE(ncclCommGetAsyncError(comm, &async) == ncclSuccess && async == ncclSuccess);
    // one set-up per communicator, one plan for the one buffer key, every call reached the kernel
    REQUIRE(gSetups == 1 && gPlans == 1 && gLaunches == 1 + kCaptured);
    if (rank == 0)
      std::printf("rank 0: %zu bytes per rank, %.3f ms per AllGather in the graph\n", bytes, ms / kCaptured);
    REQUIRE(hipGraphExecDestroy(exec) == hipSuccess && hipGraphDestroy(graph) == hipSuccess);
  }
  REQUIRE(ncclCommDestroy(comm) == ncclSuccess);
  REQUIRE(hipFree(send) == hipSuccess);
  if (mode == "uncached")
    REQUIRE(mscclppAmdFree(recv) == 0);
  else
    REQUIRE(hipFree(recv) == hipSuccess);
  registry->reset();
  std::printf("rank %d %s\n", rank, mode == "refuse" ? "refused OK" : "OK");
  std::fflush(stdout);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 3 || std::string(argv[1]) != "gpu") {
    std::fprintf(stderr, "usage: %s gpu <nranks> [floats per rank] [cached | uncached | refuse | direct]\n", argv[0]);
    return 2;
  }
  const int n = std::atoi(argv[2]);
  const size_t count = argc >= 4 ? (size_t)std::atoll(argv[3]) : (size_t)1 << 20;
  const std::string mode = argc >= 5 ? argv[4] : "cached";
  if (n < 2 || (mode != "cached" && mode != "uncached" && mode != "refuse" && mode != "direct")) return 2;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return 1;
  std::vector<pid_t> kids;
  for (int r = 0; r < n; ++r) {
    const pid_t pid = fork();
    if (pid < 0) return 1;
    if (pid == 0) std::_Exit(runRank(r, n, id, count, mode));
    kids.push_back(pid);
  }
  int failed = 0;
  for (pid_t pid : kids) {
    int st = 0;
    waitpid(pid, &st, 0);
    failed += !(WIFEXITED(st) && WEXITSTATUS(st) == 0);
  }
  std::printf(failed ? "gpu FAILED\n" : "gpu OK\n");
  return failed ? 1 : 0;
}
