// The reference's worked plugin example, examples/customized-collective-algorithm/
// customized_allgather.cu:53-271, on this library: a user AlgorithmBuilder whose algorithm builds
// PortChannels through ProxyService (connect, registerMemory / sendMemory / recvMemory,
// buildAndAddSemaphore, addMemory, portChannel), a user selector registered before
// ncclCommInitRank, and ncclAllGather reaching the user's kernel -- direct calls and a captured
// HIP graph of calls.  Every rank's output is checked exactly.  The kernel and the host-side API calls
// keep the example's spellings (namespace alias; HIP instead of CUDA runtime names).
//
//   test_customized_allgather gpu <nranks> [floats per rank] [cached | uncached | refuse]
//
// The PortChannel destination contract: `cached` (default, the example's
// cudaMalloc -> hipMalloc) is exact -- the receiving kernel only signals, the data is read after it
// -- and ProxyService warns once that the destination is cached device memory; `uncached` allocates
// the receive buffer from the uncached pool (no warning); `refuse` runs with
// MSCCLPP_AMD_PORT_CHANNEL_DST=strict and expects the first ncclAllGather to return
// ncclInvalidUsage on every rank (ProxyService::addMemory refuses the peer's buffer before any
// semaphore is built, so no rank is left waiting for another).
#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

#include "mscclpp_amd/algorithm.hpp"
#include "mscclpp_amd/core.hpp"
#include "mscclpp_amd/gpu_utils.hpp"
#include "mscclpp_amd/mscclpp_amd.h"
#include "mscclpp_amd/nccl.h"
#include "mscclpp_amd/port_channel.hpp"

namespace mscclpp = mscclpp_amd;

#define WARP_SIZE 64

#define CHECK(cond)                                                               \
  do {                                                                            \
    if (!(cond)) {                                                                \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)
#define HIP_OK(cmd) CHECK((cmd) == hipSuccess)

__global__ void __launch_bounds__(1024)
    allgather(mscclpp::DeviceHandle<mscclpp::PortChannel>* portChannels, int rank, size_t nbytesPerGPU) {
  int warpId = threadIdx.x / WARP_SIZE;
  // Each warp is responsible for one of the remote ranks
  mscclpp::DeviceHandle<mscclpp::PortChannel> portChan = portChannels[warpId];
  // sender role: put this rank's data into the peer's output at rank * nbytesPerGPU
  if (threadIdx.x % WARP_SIZE == 0) portChan.putWithSignal(rank * nbytesPerGPU, 0, nbytesPerGPU);
  __syncthreads();
  // push a sync and wait for it: the data is at the peer
  if (threadIdx.x % WARP_SIZE == 0) portChan.flush();
  // receiver role: the peer's data is in this rank's output
  if (threadIdx.x % WARP_SIZE == 0) portChan.wait();
}

struct Context {
  int rank;
  int worldSize;
  int nRanksPerNode;
  std::vector<mscclpp::RegisteredMemory> registeredMemories;
  std::shared_ptr<mscclpp::DeviceHandle<mscclpp::PortChannel>> portChannelDeviceHandles;
};

static int gInits = 0, gContexts = 0, gCalls = 0;

class AllgatherAlgoBuilder : public mscclpp::AlgorithmBuilder {
 public:
  AllgatherAlgoBuilder() = default;
  ~AllgatherAlgoBuilder() {
    if (proxyService_) proxyService_->stopProxy();
  }

  std::shared_ptr<mscclpp::Algorithm> build() override {
    auto self = std::make_shared<AllgatherAlgoBuilder>();
    std::shared_ptr<mscclpp::Algorithm> allgatherAlgo = std::make_shared<mscclpp::NativeAlgorithm>(
        "allgather", "allgather", [self](std::shared_ptr<mscclpp::Communicator> comm) { self->initialize(comm); },
        [self](const std::shared_ptr<void> ctx, const void* input, void* output, size_t inputSize, size_t outputSize,
               mscclpp::DataType dtype, mscclpp::ReduceOp op, hipStream_t stream, int nBlocks, int nThreadsPerBlock,
               const std::unordered_map<std::string, uintptr_t>& extras, mscclpp::DataType accumDtype) {
          return self->allgatherKernelFunc(ctx, input, output, inputSize, stream);
        },
        [self](std::shared_ptr<mscclpp::Communicator> comm, const void* input, void* output, size_t inputSize,
               size_t outputSize,
               mscclpp::DataType dtype) { return self->initAllgatherContext(comm, input, output, inputSize, dtype); },
        [self](const void* input, void* output, size_t inputSize, size_t outputSize, mscclpp::DataType dtype,
               bool symmetricMemory) {
          return self->generateAllgatherContextKey(input, output, inputSize, outputSize, dtype, symmetricMemory);
        });
    return allgatherAlgo;
  }

 private:
  std::vector<mscclpp::Connection> conns_;
  std::shared_ptr<mscclpp::ProxyService> proxyService_;
  int worldSize_ = 0;

  void initialize(std::shared_ptr<mscclpp::Communicator> comm) {
    gInits++;
    std::vector<std::shared_future<mscclpp::Connection>> connectionFutures;
    worldSize_ = comm->bootstrap()->getNranks();
    for (int i = 0; i < worldSize_; i++) {
      if (i == comm->bootstrap()->getRank()) continue;
      connectionFutures.push_back(comm->connect(mscclpp::Transport::CudaIpc, i));
    }
    std::vector<mscclpp::Connection> connections;
    std::transform(connectionFutures.begin(), connectionFutures.end(), std::back_inserter(connections),
                   [](const auto& future) { return future.get(); });
    this->conns_ = std::move(connections);
    proxyService_ = std::make_shared<mscclpp::ProxyService>();
    proxyService_->startProxy();
  }

  mscclpp::CommResult allgatherKernelFunc(const std::shared_ptr<void> ctx, const void* input, void* output,
                                          size_t inputSize, hipStream_t stream) {
    gCalls++;
    auto algoCtx = std::static_pointer_cast<Context>(ctx);
    int rank = algoCtx->rank;
    int worldSize = algoCtx->worldSize;
    int nThreadsPerBlock = (worldSize - 1) * WARP_SIZE;
    hipLaunchKernelGGL(allgather, dim3(1), dim3(nThreadsPerBlock), 0, stream, algoCtx->portChannelDeviceHandles.get(),
                       rank, inputSize);
    if (hipGetLastError() == hipSuccess) return mscclpp::CommResult::CommSuccess;
    return mscclpp::CommResult::CommInternalError;
  }

  std::shared_ptr<void> initAllgatherContext(std::shared_ptr<mscclpp::Communicator> comm, const void* input,
                                             void* output, size_t inputSize, mscclpp::DataType dtype) {
    gContexts++;
    auto ctx = std::make_shared<Context>();
    ctx->rank = comm->bootstrap()->getRank();
    ctx->worldSize = comm->bootstrap()->getNranks();
    ctx->nRanksPerNode = comm->bootstrap()->getNranksPerNode();

    // register memories
    mscclpp::RegisteredMemory inputBufRegMem =
        comm->registerMemory((void*)input, inputSize, mscclpp::Transport::CudaIpc);
    mscclpp::RegisteredMemory outputBufRegMem =
        comm->registerMemory(output, inputSize * ctx->worldSize, mscclpp::Transport::CudaIpc);
    std::vector<std::shared_future<mscclpp::RegisteredMemory>> remoteRegMemories;
    for (int i = 0; i < ctx->worldSize; i++) {
      if (i == ctx->rank) continue;
      comm->sendMemory(outputBufRegMem, i, 0);
      remoteRegMemories.push_back(comm->recvMemory(i, 0));
    }

    // setup channels
    std::vector<mscclpp::DeviceHandle<mscclpp::PortChannel>> portChannels;
    mscclpp::MemoryId inputMemoryId = this->proxyService_->addMemory(inputBufRegMem);
    for (size_t i = 0; i < this->conns_.size(); i++) {
      auto remoteMemory = remoteRegMemories[i].get();
      mscclpp::MemoryId remoteMemoryId = this->proxyService_->addMemory(remoteMemory);
      portChannels.push_back(mscclpp::deviceHandle(this->proxyService_->portChannel(
          this->proxyService_->buildAndAddSemaphore(*comm, this->conns_[i]), remoteMemoryId, inputMemoryId)));
    }
    ctx->portChannelDeviceHandles =
        mscclpp::detail::gpuCallocShared<mscclpp::DeviceHandle<mscclpp::PortChannel>>(portChannels.size());
    mscclpp::gpuMemcpy(ctx->portChannelDeviceHandles.get(), portChannels.data(), portChannels.size(),
                       hipMemcpyHostToDevice);

    // keep registered memory references
    std::transform(remoteRegMemories.begin(), remoteRegMemories.end(), std::back_inserter(ctx->registeredMemories),
                   [](const auto& fut) { return fut.get(); });
    ctx->registeredMemories.push_back(inputBufRegMem);
    ctx->registeredMemories.push_back(outputBufRegMem);
    return ctx;
  }

  mscclpp::AlgorithmCtxKey generateAllgatherContextKey(const void* input, void* output, size_t inputSize,
                                                       size_t outputSize, mscclpp::DataType, bool) {
    return {(void*)input, output, inputSize, outputSize, 0};
  }
};

static int worker(int rank, int worldSize, ncclUniqueId id, size_t size, const std::string& mode) {
  const int iter = 10;
  int ndev = 0;
  HIP_OK(hipGetDeviceCount(&ndev));
  HIP_OK(hipSetDevice(rank % ndev));

  // register the algorithm and the selector before ncclCommInitRank (customized_allgather.cu:206-218)
  auto allgatherAlgoBuilder = std::make_shared<AllgatherAlgoBuilder>();
  auto algoCollectionBuilder = mscclpp::collective::AlgorithmCollectionBuilder::getInstance();
  algoCollectionBuilder->addAlgorithmBuilder(allgatherAlgoBuilder);
  algoCollectionBuilder->setAlgorithmSelector(
      [](const std::unordered_map<std::string, std::unordered_map<std::string, std::shared_ptr<mscclpp::Algorithm>>>&
             algoMapByCollective,
         const mscclpp::CollectiveRequest& request) -> std::shared_ptr<mscclpp::Algorithm> {
        if (request.collective != "allgather") return nullptr;
        return algoMapByCollective.at(request.collective).at("allgather");
      });

  float *sendbuff, *recvbuff;
  hipStream_t stream;
  HIP_OK(hipMalloc(&sendbuff, size * sizeof(float)));
  if (mode == "uncached")
    CHECK(mscclppAmdMallocUncached((void**)&recvbuff, size * sizeof(float) * worldSize) == 0);
  else
    HIP_OK(hipMalloc(&recvbuff, size * sizeof(float) * worldSize));
  if (mode == "refuse") setenv("MSCCLPP_AMD_PORT_CHANNEL_DST", "strict", 1);
  std::vector<float> h(size);
  for (size_t i = 0; i < size; ++i) h[i] = (float)(rank * 1000003 + (int)(i % 999983));
  HIP_OK(hipMemcpy(sendbuff, h.data(), size * sizeof(float), hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(recvbuff + rank * size, sendbuff, size * sizeof(float), hipMemcpyDeviceToDevice));
  HIP_OK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));

  ncclComm_t comm;
  CHECK(ncclCommInitRank(&comm, worldSize, id, rank) == ncclSuccess);
  auto check = [&](const char* what) {
    std::vector<float> out(size * worldSize);
    HIP_OK(hipMemcpy(out.data(), recvbuff, out.size() * sizeof(float), hipMemcpyDeviceToHost));
    for (int r = 0; r < worldSize; ++r)
      for (size_t i = 0; i < size; ++i)
        if (out[r * size + i] != (float)(r * 1000003 + (int)(i % 999983))) {
          std::fprintf(stderr, "rank %d %s: element %zu of rank %d's block wrong\n", rank, what, i, r);
          std::exit(1);
        }
  };
  if (mode == "refuse") {  // the context's portChannel() refuses the cached destination
    const ncclResult_t r = ncclAllGather(sendbuff, recvbuff, size, ncclFloat, comm, stream);
    CHECK(r == ncclInvalidUsage);
    CHECK(std::string(ncclGetLastError(comm)).find("cached device memory") != std::string::npos);
    CHECK(ncclCommDestroy(comm) == ncclSuccess);
    HIP_OK(hipFree(sendbuff));
    HIP_OK(hipFree(recvbuff));
    algoCollectionBuilder->reset();
    std::printf("rank %d refused OK\n", rank);
    std::fflush(stdout);
    return 0;
  }
  // direct calls (the first one builds the context)
  CHECK(ncclAllGather(sendbuff, recvbuff, size, ncclFloat, comm, stream) == ncclSuccess);
  HIP_OK(hipStreamSynchronize(stream));
  check("first call");
  HIP_OK(hipMemset(recvbuff, 0, size * sizeof(float) * worldSize));
  HIP_OK(hipMemcpy(recvbuff + rank * size, sendbuff, size * sizeof(float), hipMemcpyDeviceToDevice));
  mscclppAmdCommBarrier(comm);
  // a captured graph of `iter` calls (customized_allgather.cu:233-250)
  hipGraph_t graph;
  hipGraphExec_t graphExec;
  HIP_OK(hipStreamBeginCapture(stream, hipStreamCaptureModeGlobal));
  for (int i = 0; i < iter; ++i) CHECK(ncclAllGather(sendbuff, recvbuff, size, ncclFloat, comm, stream) == ncclSuccess);
  HIP_OK(hipStreamEndCapture(stream, &graph));
  HIP_OK(hipGraphInstantiate(&graphExec, graph, nullptr, nullptr, 0));
  hipEvent_t start, end;
  HIP_OK(hipEventCreate(&start));
  HIP_OK(hipEventCreate(&end));
  HIP_OK(hipDeviceSynchronize());
  HIP_OK(hipEventRecord(start, stream));
  HIP_OK(hipGraphLaunch(graphExec, stream));
  HIP_OK(hipEventRecord(end, stream));
  HIP_OK(hipEventSynchronize(end));
  float ms = 0;
  HIP_OK(hipEventElapsedTime(&ms, start, end));
  check("graph");
  ncclResult_t async = ncclSuccess;
  CHECK(ncclCommGetAsyncError(comm, &async) == ncclSuccess && async == ncclSuccess);
  CHECK(gInits == 1 && gContexts == 1 && gCalls == 1 + iter);
  if (rank == 0)
    std::printf("rank 0: %zu bytes per rank, %.3f ms/iter, %.2f GB/s\n", size * sizeof(float), ms / iter,
                (double)size * sizeof(float) * (worldSize - 1) / (ms / iter) * 1e-6);
  HIP_OK(hipGraphExecDestroy(graphExec));
  HIP_OK(hipGraphDestroy(graph));
  CHECK(ncclCommDestroy(comm) == ncclSuccess);
  HIP_OK(hipFree(sendbuff));
  if (mode == "uncached")
    CHECK(mscclppAmdFree(recvbuff) == 0);
  else
    HIP_OK(hipFree(recvbuff));
  algoCollectionBuilder->reset();
  std::printf("rank %d OK\n", rank);
  std::fflush(stdout);
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 3 && std::string(argv[1]) == "gpu") {
    const int n = std::atoi(argv[2]);
    const size_t size = argc >= 4 ? (size_t)std::atoll(argv[3]) : (size_t)1 << 20;
    const std::string mode = argc >= 5 ? argv[4] : "cached";
    if (mode != "cached" && mode != "uncached" && mode != "refuse") return 2;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return 1;
    std::vector<pid_t> pids;
    for (int r = 0; r < n; ++r) {
      pid_t pid = fork();
      if (pid < 0) return 1;
      if (pid == 0) std::_Exit(worker(r, n, id, size, mode));
      pids.push_back(pid);
    }
    int bad = 0;
    for (pid_t pid : pids) {
      int st = 0;
      waitpid(pid, &st, 0);
      if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) bad++;
    }
    std::printf(bad ? "gpu FAILED\n" : "gpu OK\n");
    return bad ? 1 : 0;
  }
  std::fprintf(stderr, "usage: %s gpu <nranks> [floats per rank]\n", argv[0]);
  return 2;
}
