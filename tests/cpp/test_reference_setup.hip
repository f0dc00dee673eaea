// The reference's user-level setup sequence, written only with its spellings (<mscclpp/...> headers,
// namespace mscclpp, TcpBootstrap, Communicator(bootstrap), EndpointConfig{transport, {DeviceType,
// id}}, GpuBuffer, DeviceSyncer), run on this library.  Six modes:
//
//   local       one rank: a PortChannel from one GpuBuffer to another over a connection to itself,
//               one workgroup writes and puts with a signal, another waits and checks
//               (the sequence of test/unit/local_channel_tests.cu:15-78)
//   pair PORT   two processes meet at 127.0.0.1:PORT through TcpBootstrap::initialize("ip:port"),
//               build a MemoryChannel and a packet MemoryChannel over GpuBuffers, and run a
//               bidirectional put (+ signal / wait), get and putPackets / unpackPackets round, each
//               checked word by word (the sequence of examples/tutorials/03-memory-channel)
//   uid         the parent creates a UniqueId (TcpBootstrap::createUniqueId); two forked ranks
//               initialize with it, and their Communicators exchange a buffer through a memory
//               channel
//   context     one process, no communicator: Context::create, two endpoints (GPU 0 and GPU 1, or
//               GPU 0 twice on a one-GPU box), Context::connect both ways, SemaphoreStub per side,
//               Semaphore(localStub, remoteStub), BaseMemoryChannel -- and the relaxedSignal /
//               relaxedWait ping-pong of examples/tutorials/01-basic-concepts, which must take at
//               least the spin the waiting side adds per round, and leave both tokens at `iter`
//   port PORT   the port-channel tutorial (examples/tutorials/04-port-channel): ProxyService::addSemaphore
//               of a Communicator-built semaphore, portChannel(semaId, remote, local), a one-thread
//               kernel doing signal / wait / putWithSignal / wait captured 20 times into a HIP graph
//               per size (1 KiB, 1 MiB, 16 MiB) with the proxy stopped during capture and restarted
//               for the replays, the peer's half checked after each size
//   executor PLAN   the sequence of test/executor_test.cc: a UniqueId from the parent, two ranks with
//               TcpBootstrap + Communicator + Executor + ExecutionPlan(PLAN, rank) + GpuBuffer, an
//               in-place fp16 AllReduce through Executor::execute with PacketType::LL16 and ::LL8,
//               three calls each on fresh inputs whose sums are exact
// Exit status 0 and "<mode> OK" on success.
#include <hip/hip_runtime.h>
#include <signal.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <mscclpp/atomic_device.hpp>
#include <mscclpp/concurrency_device.hpp>
#include <mscclpp/core.hpp>
#include <mscclpp/env.hpp>
#include <mscclpp/errors.hpp>
#include <mscclpp/executor.hpp>
#include <mscclpp/gpu_utils.hpp>
#include <mscclpp/memory_channel.hpp>
#include <mscclpp/memory_channel_device.hpp>
#include <mscclpp/numa.hpp>
#include <mscclpp/poll_device.hpp>
#include <mscclpp/port_channel.hpp>
#include <mscclpp/port_channel_device.hpp>
#include <mscclpp/utils.hpp>

#define CHECK(cond)                                                               \
  do {                                                                            \
    if (!(cond)) {                                                                \
      std::fprintf(stderr, "%s:%d check failed: %s\n", __FILE__, __LINE__, #cond); \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

constexpr int kMagic = 777;

// ---- local: PortChannel loopback -------------------------------------------------------------------
__constant__ mscclpp::PortChannelDeviceHandle gPortChannel;

__global__ void localPortChannelKernel(int* dst, int* src, size_t bytes, int* ret) {
  if (blockIdx.x == 0) {
    for (size_t i = threadIdx.x; i < bytes / sizeof(int); i += blockDim.x) src[i] = kMagic;
    __syncthreads();
    if (threadIdx.x == 0) gPortChannel.putWithSignal(0, bytes);
  } else {
    if (threadIdx.x == 0) gPortChannel.wait();
    __syncthreads();
    for (size_t i = threadIdx.x; i < bytes / sizeof(int); i += blockDim.x)
      if (dst[i] != kMagic) *ret = 1;
  }
}

__global__ void loopbackPutWaitKernel(size_t bytes) {
  gPortChannel.putWithSignal(0, bytes);
  gPortChannel.wait();
}

static int runLocal() {
  MSCCLPP_CUDATHROW(hipSetDevice(0));
  auto bootstrap = std::make_shared<mscclpp::TcpBootstrap>(/*rank*/ 0, /*nRanks*/ 1);
  bootstrap->initialize(mscclpp::TcpBootstrap::createUniqueId());
  auto communicator = std::make_shared<mscclpp::Communicator>(bootstrap);
  const mscclpp::Transport transport = mscclpp::Transport::CudaIpc;
  auto connection = communicator->connect(transport, /*remoteRank*/ 0).get();

  const size_t bytes = 4 << 20;
  auto srcBuff = mscclpp::GpuBuffer(bytes).memory();
  auto dstBuff = mscclpp::GpuBuffer(bytes).memory();
  auto srcMem = communicator->registerMemory(srcBuff.get(), bytes, transport);
  auto dstMem = communicator->registerMemory(dstBuff.get(), bytes, transport);

  auto proxyService = std::make_shared<mscclpp::ProxyService>();
  auto srcMemId = proxyService->addMemory(srcMem);
  auto dstMemId = proxyService->addMemory(dstMem);
  auto sid = proxyService->buildAndAddSemaphore(*communicator, connection);
  auto portChannel = proxyService->portChannel(sid, dstMemId, srcMemId);
  auto handle = portChannel.deviceHandle();
  MSCCLPP_CUDATHROW(hipMemcpyToSymbol(HIP_SYMBOL(gPortChannel), &handle, sizeof(handle)));

  std::shared_ptr<int> ret = mscclpp::detail::gpuCallocHostShared<int>();
  proxyService->startProxy();
  hipLaunchKernelGGL(localPortChannelKernel, dim3(2), dim3(1024), 0, 0, (int*)dstBuff.get(), (int*)srcBuff.get(),
                     bytes, ret.get());
  MSCCLPP_CUDATHROW(hipDeviceSynchronize());
  CHECK(*ret == 0);
  // One process, one proxy, the GPU to itself: 1000 graph-replayed iterations of putWithSignal +
  // wait through the loopback channel (the 2-rank port mode's shape with no second process on the
  // device), so DESIGN.md §9 can tell the proxy path's own latency from cross-process scheduling.
  hipStream_t stream;
  MSCCLPP_CUDATHROW(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  const int iter = 1000;
  for (size_t copyBytes : {(size_t)1024, (size_t)1 << 20}) {
    hipGraph_t graph;
    hipGraphExec_t exec;
    MSCCLPP_CUDATHROW(hipStreamBeginCapture(stream, hipStreamCaptureModeGlobal));
    for (int i = 0; i < iter; ++i) hipLaunchKernelGGL(loopbackPutWaitKernel, dim3(1), dim3(1), 0, stream, copyBytes);
    MSCCLPP_CUDATHROW(hipStreamEndCapture(stream, &graph));
    MSCCLPP_CUDATHROW(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    MSCCLPP_CUDATHROW(hipGraphLaunch(exec, stream));  // warm
    MSCCLPP_CUDATHROW(hipStreamSynchronize(stream));
    hipEvent_t t0, t1;
    MSCCLPP_CUDATHROW(hipEventCreate(&t0));
    MSCCLPP_CUDATHROW(hipEventCreate(&t1));
    MSCCLPP_CUDATHROW(hipEventRecord(t0, stream));
    MSCCLPP_CUDATHROW(hipGraphLaunch(exec, stream));
    MSCCLPP_CUDATHROW(hipEventRecord(t1, stream));
    MSCCLPP_CUDATHROW(hipStreamSynchronize(stream));
    float ms = 0;
    MSCCLPP_CUDATHROW(hipEventElapsedTime(&ms, t0, t1));
    std::printf("LOCAL_JSON {\"bytes\": %zu, \"us_per_iter\": %.3f, \"iters\": %d}\n", copyBytes, ms * 1e3 / iter,
                iter);
    MSCCLPP_CUDATHROW(hipEventDestroy(t0));
    MSCCLPP_CUDATHROW(hipEventDestroy(t1));
    MSCCLPP_CUDATHROW(hipGraphExecDestroy(exec));
    MSCCLPP_CUDATHROW(hipGraphDestroy(graph));
  }
  MSCCLPP_CUDATHROW(hipStreamDestroy(stream));
  proxyService->stopProxy();
  std::printf("local OK\n");
  return 0;
}

// ---- pair: the memory-channel tutorial's three kernels ------------------------------------------
__device__ mscclpp::DeviceSyncer devSyncer;

__global__ void bidirPutKernel(mscclpp::MemoryChannelDeviceHandle* ch, size_t copyBytes, int myRank) {
  const int tid = threadIdx.x + blockIdx.x * blockDim.x;
  if (tid == 0) {
    ch->relaxedSignal();
    ch->relaxedWait();
  }
  devSyncer.sync(gridDim.x);
  const uint64_t off = myRank * copyBytes;
  ch->put(off, off, copyBytes, tid, blockDim.x * gridDim.x);
  devSyncer.sync(gridDim.x);
  if (tid == 0) {
    ch->signal();
    ch->wait();
  }
}

__global__ void bidirGetKernel(mscclpp::MemoryChannelDeviceHandle* ch, size_t copyBytes, int myRank) {
  const int tid = threadIdx.x + blockIdx.x * blockDim.x;
  if (tid == 0) {
    ch->relaxedSignal();
    ch->relaxedWait();
  }
  devSyncer.sync(gridDim.x);
  const uint64_t off = (myRank ^ 1) * copyBytes;
  ch->get(off, off, copyBytes, tid, blockDim.x * gridDim.x);
  devSyncer.sync(gridDim.x);
  if (tid == 0) {  // the peer may not overwrite what this rank still reads
    ch->signal();
    ch->wait();
  }
}

__global__ void bidirPutPacketKernel(mscclpp::MemoryChannelDeviceHandle* ch, size_t copyBytes, int myRank,
                                     uint32_t flag) {
  const int tid = threadIdx.x + blockIdx.x * blockDim.x;
  if (tid == 0) {
    ch->relaxedSignal();
    ch->relaxedWait();
  }
  devSyncer.sync(gridDim.x);
  const uint64_t off = myRank * copyBytes;
  ch->putPackets(0, off, copyBytes, tid, blockDim.x * gridDim.x, flag);
  ch->unpackPackets(0, off, copyBytes, tid, blockDim.x * gridDim.x, flag);
}

// Watchdog over one timed graph of a pair rank: if the graph has not completed after `seconds`, it
// prints what the rank's waits see -- the device error record, this module's DeviceSyncer words
// (count, generation, timed out) and the channel's inbound / expected tokens, copied on a stream of
// its own into pinned words allocated up front -- and ends the rank (exit 3), so a stall names its
// wait instead of running into the test's timeout.
struct GraphWatchdog {
  std::mutex mu;
  std::condition_variable cv;
  bool done = false;
  std::thread th;
  GraphWatchdog(int rank, const char* what, size_t bytes, int seconds, hipStream_t diag, uint32_t* pinned,
                const void* err, const void* syncer, const void* inbound, const void* expected) {
    th = std::thread([this, rank, what, bytes, seconds, diag, pinned, err, syncer, inbound, expected] {
      {
        std::unique_lock<std::mutex> lk(mu);
        if (cv.wait_for(lk, std::chrono::seconds(seconds), [this] { return done; })) return;
      }
      std::memset(pinned, 0xFF, 12 * sizeof(uint32_t));
      bool ok = hipMemcpyAsync(pinned, err, 16, hipMemcpyDeviceToHost, diag) == hipSuccess &&
                hipMemcpyAsync(pinned + 4, syncer, 12, hipMemcpyDeviceToHost, diag) == hipSuccess &&
                hipMemcpyAsync(pinned + 8, inbound, 8, hipMemcpyDeviceToHost, diag) == hipSuccess &&
                hipMemcpyAsync(pinned + 10, expected, 8, hipMemcpyDeviceToHost, diag) == hipSuccess;
      const auto t0 = std::chrono::steady_clock::now();
      while (ok && hipStreamQuery(diag) == hipErrorNotReady)
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) ok = false;
      uint64_t in = 0, ex = 0;
      std::memcpy(&in, pinned + 8, 8);
      std::memcpy(&ex, pinned + 10, 8);
      std::printf("rank %d [%s] bytes %zu: graph not done after %d s; error %u (flag %u, byte %u, seen %u); "
                  "DeviceSyncer count %u gen %u timedOut %u; inbound token %llu, expected %llu%s\n",
                  rank, what, bytes, seconds, pinned[0], pinned[1], pinned[2], pinned[3], pinned[4], pinned[5],
                  pinned[6], (unsigned long long)in, (unsigned long long)ex, ok ? "" : " (diagnostic copy incomplete)");
      std::fflush(stdout);
      std::_Exit(3);
    });
  }
  ~GraphWatchdog() {
    {
      std::lock_guard<std::mutex> lk(mu);
      done = true;
    }
    cv.notify_all();
    th.join();
  }
};

static std::vector<int> pattern(int rank, size_t n, int round) {
  std::vector<int> v(n);
  for (size_t i = 0; i < n; ++i) v[i] = (rank + 1) * 1000003 + (int)i * 7 + round * 31;
  return v;
}

static int pairWorker(int myRank, const std::string& ipPort) {
  MSCCLPP_CUDATHROW(hipSetDevice(0));
  int gpuId = 0;
  MSCCLPP_CUDATHROW(hipGetDevice(&gpuId));
  const int remoteRank = myRank ^ 1, nRanks = 2;
  const mscclpp::Transport transport = mscclpp::Transport::CudaIpc;
  const size_t copyBytes = 1 << 20, n = copyBytes / sizeof(int);
  const size_t maxBytes = (size_t)128 << 20;  // the tutorial's largest size (bidir_memory_channel.cu:173)

  auto bootstrap = std::make_shared<mscclpp::TcpBootstrap>(myRank, nRanks);
  bootstrap->initialize(ipPort);
  mscclpp::Communicator comm(bootstrap);
  auto conn = comm.connect({transport, {mscclpp::DeviceType::GPU, gpuId}}, remoteRank).get();
  auto sema = comm.buildSemaphore(conn, remoteRank).get();

  mscclpp::GpuBuffer buffer(2 * maxBytes);
  mscclpp::GpuBuffer pktBuffer(4 * maxBytes);
  CHECK(buffer.bytes() == 2 * maxBytes && buffer.deviceId() == gpuId);
  auto localRegMem = comm.registerMemory(buffer.data(), buffer.bytes(), transport);
  auto localPktRegMem = comm.registerMemory(pktBuffer.data(), pktBuffer.bytes(), transport);
  comm.sendMemory(localRegMem, remoteRank);
  comm.sendMemory(localPktRegMem, remoteRank);
  auto remoteRegMemFuture = comm.recvMemory(remoteRank);
  auto remotePktRegMemFuture = comm.recvMemory(remoteRank);
  mscclpp::RegisteredMemory remoteRegMem = remoteRegMemFuture.get();
  mscclpp::RegisteredMemory remotePktRegMem = remotePktRegMemFuture.get();

  // Both channels on ONE MemoryDevice2DeviceSemaphore.  The tutorial builds each from the Semaphore
  // (bidir_memory_channel.cu:128-130), and a MemoryChannel made from a Semaphore gets a device
  // semaphore of its own (memory_channel.cc:25-27 -> semaphore.cc:216-217): two expected counters over
  // one inbound token.  After the put / get kernels' 12,000 signals, the packet kernel's handshake
  // then passes without waiting, and a rank that starts launch f + 1 overwrites packets its peer is
  // still unpacking for flag f -- seen here at 128 MiB (round 6): rank 1 waiting for flag 2012 at a
  // packet that already held 2013, rank 0 waiting for 2013.  Sharing the device semaphore (the
  // reference's other constructor, memory_channel.cc:17-19) keeps one counter, as the tutorial means.
  auto d2dSema = std::make_shared<mscclpp::MemoryDevice2DeviceSemaphore>(sema);
  mscclpp::MemoryChannel memChan(d2dSema, /*dst*/ remoteRegMem, /*src*/ localRegMem);
  mscclpp::MemoryChannel memPktChan(d2dSema, /*dst*/ remotePktRegMem, /*src*/ localRegMem,
                                    /*packetBuffer*/ localPktRegMem.data());
  auto h = memChan.deviceHandle();
  auto hp = memPktChan.deviceHandle();
  // the semantics above, as the reference has them: channels on one device semaphore share its
  // expected counter; a channel made from the Semaphore itself has a counter of its own over the
  // same inbound token
  CHECK(h.semaphore_.expectedInboundToken == hp.semaphore_.expectedInboundToken);
  {
    mscclpp::MemoryChannel own(sema, remoteRegMem, localRegMem);
    const auto ho = own.deviceHandle();
    CHECK(ho.semaphore_.inboundToken == h.semaphore_.inboundToken);
    CHECK(ho.semaphore_.expectedInboundToken != h.semaphore_.expectedInboundToken);
  }
  auto dh = mscclpp::detail::gpuCallocShared<mscclpp::MemoryChannelDeviceHandle>();
  auto dhp = mscclpp::detail::gpuCallocShared<mscclpp::MemoryChannelDeviceHandle>();
  mscclpp::gpuMemcpy(dh.get(), &h, 1, hipMemcpyHostToDevice);
  mscclpp::gpuMemcpy(dhp.get(), &hp, 1, hipMemcpyHostToDevice);
  hipStream_t stream;
  MSCCLPP_CUDATHROW(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  int* buf = (int*)buffer.data();
  std::vector<int> got(2 * n);

  auto fillMine = [&](int round) {
    auto mine = pattern(myRank, n, round);
    std::vector<int> zeros(n, 0);
    mscclpp::gpuMemcpy(buf + myRank * n, mine.data(), n, hipMemcpyHostToDevice);
    mscclpp::gpuMemcpy(buf + remoteRank * n, zeros.data(), n, hipMemcpyHostToDevice);
    MSCCLPP_CUDATHROW(hipDeviceSynchronize());
    bootstrap->barrier();
  };
  auto expectAt = [&](int region, int ofRank, int round, const char* what) {
    mscclpp::gpuMemcpy(got.data(), buf, 2 * n, hipMemcpyDeviceToHost);
    const auto want = pattern(ofRank, n, round);
    size_t bad = 0;
    for (size_t i = 0; i < n; ++i) bad += got[region * n + i] != want[i];
    if (bad) std::fprintf(stderr, "rank %d %s: %zu of %zu words wrong\n", myRank, what, bad, n);
    CHECK(bad == 0);
  };

  // put: my region goes to the peer's buffer at the same offset
  fillMine(0);
  hipLaunchKernelGGL(bidirPutKernel, dim3(32), dim3(1024), 0, stream, dh.get(), copyBytes, myRank);
  MSCCLPP_CUDATHROW(hipStreamSynchronize(stream));
  bootstrap->barrier();
  expectAt(remoteRank, remoteRank, 0, "put");
  expectAt(myRank, myRank, 0, "put (own region)");

  // get: the peer's region is read from the peer's buffer
  fillMine(1);
  hipLaunchKernelGGL(bidirGetKernel, dim3(32), dim3(1024), 0, stream, dh.get(), copyBytes, myRank);
  MSCCLPP_CUDATHROW(hipStreamSynchronize(stream));
  bootstrap->barrier();
  expectAt(remoteRank, remoteRank, 1, "get");

  // packets: my region goes to the peer's packet buffer; I unpack the peer's into my own region
  for (uint32_t flag = 1; flag <= 3; ++flag) {
    fillMine(10 + (int)flag);
    hipLaunchKernelGGL(bidirPutPacketKernel, dim3(32), dim3(1024), 0, stream, dhp.get(), copyBytes, myRank, flag);
    MSCCLPP_CUDATHROW(hipStreamSynchronize(stream));
    bootstrap->barrier();
    expectAt(myRank, remoteRank, 10 + (int)flag, "putPackets/unpackPackets");
  }

  // the tutorial's timing (bidir_memory_channel.cu:170-210): 1000 graph-captured launches per kernel
  // and size, one event pair on rank 0, its own log line; packet flags keep counting from 4, one per
  // captured launch.  (This get kernel ends with one more signal / wait than the tutorial's, so the
  // peer never overwrites what a rank still reads; its rows carry that extra round trip.)
  const int iter = 1000;
  uint32_t flag = 4;
  hipStream_t diag;
  MSCCLPP_CUDATHROW(hipStreamCreateWithFlags(&diag, hipStreamNonBlocking));
  uint32_t* pinned = nullptr;
  MSCCLPP_CUDATHROW(hipHostMalloc((void**)&pinned, 64, hipHostMallocDefault));
  void* syncerAddr = nullptr;
  MSCCLPP_CUDATHROW(hipGetSymbolAddress(&syncerAddr, HIP_SYMBOL(devSyncer)));
  for (int k = 0; k < 3; ++k) {
    const char* name = k == 0 ? "Bidir Put" : k == 1 ? "Bidir Get" : "Bidir Put Packets";
    for (size_t bytes : {(size_t)1024, (size_t)1 << 20, maxBytes}) {
      hipGraph_t graph;
      hipGraphExec_t exec;
      MSCCLPP_CUDATHROW(hipStreamBeginCapture(stream, hipStreamCaptureModeGlobal));
      for (int i = 0; i < iter; ++i) {
        if (k == 0)
          hipLaunchKernelGGL(bidirPutKernel, dim3(32), dim3(1024), 0, stream, dh.get(), bytes, myRank);
        else if (k == 1)
          hipLaunchKernelGGL(bidirGetKernel, dim3(32), dim3(1024), 0, stream, dh.get(), bytes, myRank);
        else
          hipLaunchKernelGGL(bidirPutPacketKernel, dim3(32), dim3(1024), 0, stream, dhp.get(), bytes, myRank, flag++);
      }
      MSCCLPP_CUDATHROW(hipStreamEndCapture(stream, &graph));
      MSCCLPP_CUDATHROW(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
      MSCCLPP_CUDATHROW(hipDeviceSynchronize());
      bootstrap->barrier();
      hipEvent_t t0, t1;
      MSCCLPP_CUDATHROW(hipEventCreate(&t0));
      MSCCLPP_CUDATHROW(hipEventCreate(&t1));
      MSCCLPP_CUDATHROW(hipEventRecord(t0, stream));
      MSCCLPP_CUDATHROW(hipGraphLaunch(exec, stream));
      MSCCLPP_CUDATHROW(hipEventRecord(t1, stream));
      {
        const auto& sem = (k == 2 ? hp : h).semaphore_;
        GraphWatchdog wd(myRank, name, bytes, 60, diag, pinned, comm.deviceErrorWord(), syncerAddr, sem.inboundToken,
                         sem.expectedInboundToken);
        MSCCLPP_CUDATHROW(hipStreamSynchronize(stream));
      }
      // a wait that ran out of budget in any of the 1000 launches fails the run here, naming the
      // kernel, the size and the error record (code, flag, packet byte, flag seen)
      uint32_t rec[4] = {0, 0, 0, 0};
      MSCCLPP_CUDATHROW(hipMemcpy(rec, comm.deviceErrorWord(), sizeof(rec), hipMemcpyDeviceToHost));
      if (rec[0]) {
        std::printf("rank %d [%s] bytes %zu: device error %u (flag %u, byte %u, seen %u)\n", myRank, name, bytes,
                    rec[0], rec[1], rec[2], rec[3]);
        std::fflush(stdout);
      }
      CHECK(rec[0] == 0);
      if (myRank == 0) {
        float ms = 0;
        MSCCLPP_CUDATHROW(hipEventElapsedTime(&ms, t0, t1));
        const float per = ms / iter;
        std::printf("Rank %d (GPU %d): [%s] bytes %zu, elapsed %g ms/iter, BW %g GB/s\n", myRank, gpuId, name, bytes,
                    per, (float)bytes / per * 1e-6f);
        std::printf("PAIR_JSON {\"kernel\": \"%s\", \"bytes\": %zu, \"us_per_iter\": %.3f, \"GBs\": %.3f}\n", name,
                    bytes, per * 1e3, (float)bytes / per * 1e-6f);
        std::fflush(stdout);
      }
      MSCCLPP_CUDATHROW(hipEventDestroy(t0));
      MSCCLPP_CUDATHROW(hipEventDestroy(t1));
      MSCCLPP_CUDATHROW(hipGraphExecDestroy(exec));
      MSCCLPP_CUDATHROW(hipGraphDestroy(graph));
      bootstrap->barrier();
    }
  }
  MSCCLPP_CUDATHROW(hipStreamDestroy(stream));
  MSCCLPP_CUDATHROW(hipStreamDestroy(diag));
  MSCCLPP_CUDATHROW(hipHostFree(pinned));
  bootstrap->barrier();
  std::printf("rank %d pair OK\n", myRank);
  std::fflush(stdout);
  return 0;
}

// ---- uid: a UniqueId from the parent, Communicators in the children ------------------------------
__global__ void putSignalKernel(mscclpp::MemoryChannelDeviceHandle ch, size_t bytes) {
  ch.put(0, 0, bytes, threadIdx.x, blockDim.x);
  __syncthreads();
  if (threadIdx.x == 0) {
    ch.signal();
    ch.wait();
  }
}

static int uidWorker(int myRank, mscclpp::UniqueId id) {
  MSCCLPP_CUDATHROW(hipSetDevice(0));
  auto bootstrap = std::make_shared<mscclpp::TcpBootstrap>(myRank, 2);
  bootstrap->initialize(id);
  CHECK(bootstrap->getUniqueId() == id && bootstrap->getRank() == myRank && bootstrap->getNranks() == 2);
  auto comm = std::make_shared<mscclpp::Communicator>(bootstrap);
  const int remote = myRank ^ 1;
  auto conn = comm->connect(mscclpp::Transport::CudaIpc, remote).get();
  auto sema = comm->buildSemaphore(conn, remote).get();
  const size_t n = 1 << 16;
  mscclpp::GpuBuffer<int> src(n), dst(n);
  auto srcMem = comm->registerMemory(src.data(), src.bytes(), mscclpp::Transport::CudaIpc);
  auto dstMem = comm->registerMemory(dst.data(), dst.bytes(), mscclpp::Transport::CudaIpc);
  comm->sendMemory(dstMem, remote);
  auto peerDst = comm->recvMemory(remote).get();
  auto mine = pattern(myRank, n, 5);
  mscclpp::gpuMemcpy(src.data(), mine.data(), n, hipMemcpyHostToDevice);
  bootstrap->barrier();
  mscclpp::MemoryChannel ch(sema, peerDst, srcMem);
  hipLaunchKernelGGL(putSignalKernel, dim3(1), dim3(1024), 0, 0, ch.deviceHandle(), n * sizeof(int));
  MSCCLPP_CUDATHROW(hipDeviceSynchronize());
  std::vector<int> got(n);
  mscclpp::gpuMemcpy(got.data(), dst.data(), n, hipMemcpyDeviceToHost);
  CHECK(got == pattern(remote, n, 5));
  bootstrap->barrier();
  std::printf("rank %d uid OK\n", myRank);
  std::fflush(stdout);
  return 0;
}

// ---- context: two endpoints of this process ----------------------------------------------------------
__device__ void spinTicks(uint64_t ticks) {  // s_memrealtime: 100 MHz
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
  }
}

__global__ void pingKernel0(mscclpp::BaseMemoryChannelDeviceHandle* h, int iter) {
  if (threadIdx.x + blockIdx.x * blockDim.x == 0) {
    for (int i = 0; i < iter; ++i) {
      h->relaxedWait();
      spinTicks(10000);  // 100 us
      h->relaxedSignal();
    }
  }
}

__global__ void pingKernel1(mscclpp::BaseMemoryChannelDeviceHandle* h, int iter) {
  if (threadIdx.x + blockIdx.x * blockDim.x == 0) {
    for (int i = 0; i < iter; ++i) {
      h->relaxedSignal();
      h->relaxedWait();
    }
  }
}

static int runContext() {
  int ndev = 0;
  MSCCLPP_CUDATHROW(hipGetDeviceCount(&ndev));
  const int dev0 = 0, dev1 = ndev > 1 ? 1 : 0;
  const int iter = 50;
  const mscclpp::Transport transport = mscclpp::Transport::CudaIpc;
  auto ctx = mscclpp::Context::create();
  mscclpp::Endpoint ep0 = ctx->createEndpoint({transport, {mscclpp::DeviceType::GPU, dev0}});
  mscclpp::Endpoint ep1 = ctx->createEndpoint({transport, {mscclpp::DeviceType::GPU, dev1}});
  // an endpoint survives a round trip through its wire form
  const mscclpp::Endpoint ep1b = mscclpp::Endpoint::deserialize(ep1.serialize());
  CHECK(ep1b.device().id == dev1 && ep1b.pidHash() == ep1.pidHash() && ep1b.hostHash() == ep0.hostHash());

  mscclpp::Connection conn0 = ctx->connect(/*localEndpoint*/ ep0, /*remoteEndpoint*/ ep1b);
  mscclpp::SemaphoreStub semaStub0(conn0);
  mscclpp::Connection conn1 = ctx->connect(/*localEndpoint*/ ep1, /*remoteEndpoint*/ ep0);
  mscclpp::SemaphoreStub semaStub1(conn1);
  CHECK(conn0.context() == ctx && conn0.localDevice().id == dev0 && conn1.localDevice().id == dev1);

  MSCCLPP_CUDATHROW(hipSetDevice(dev0));
  mscclpp::Semaphore sema0(/*localSemaphoreStub*/ semaStub0, /*remoteSemaphoreStub*/ semaStub1);
  mscclpp::BaseMemoryChannel memChan0(sema0);
  mscclpp::BaseMemoryChannelDeviceHandle h0 = memChan0.deviceHandle();
  auto d0 = mscclpp::detail::gpuCallocShared<mscclpp::BaseMemoryChannelDeviceHandle>();
  mscclpp::gpuMemcpy(d0.get(), &h0, 1, hipMemcpyHostToDevice);
  hipStream_t s0;
  MSCCLPP_CUDATHROW(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));

  MSCCLPP_CUDATHROW(hipSetDevice(dev1));
  // the remote stub travels as bytes, as it would between processes
  mscclpp::Semaphore sema1(semaStub1, mscclpp::SemaphoreStub::deserialize(semaStub0.serialize()));
  mscclpp::BaseMemoryChannel memChan1(sema1);
  mscclpp::BaseMemoryChannelDeviceHandle h1 = memChan1.deviceHandle();
  auto d1 = mscclpp::detail::gpuCallocShared<mscclpp::BaseMemoryChannelDeviceHandle>();
  mscclpp::gpuMemcpy(d1.get(), &h1, 1, hipMemcpyHostToDevice);
  hipStream_t s1;
  MSCCLPP_CUDATHROW(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));

  MSCCLPP_CUDATHROW(hipSetDevice(dev0));
  hipLaunchKernelGGL(pingKernel0, dim3(1), dim3(1), 0, s0, d0.get(), iter);
  MSCCLPP_CUDATHROW(hipGetLastError());
  MSCCLPP_CUDATHROW(hipSetDevice(dev1));
  hipEvent_t start, end;
  MSCCLPP_CUDATHROW(hipEventCreate(&start));
  MSCCLPP_CUDATHROW(hipEventCreate(&end));
  MSCCLPP_CUDATHROW(hipEventRecord(start, s1));
  hipLaunchKernelGGL(pingKernel1, dim3(1), dim3(1), 0, s1, d1.get(), iter);
  MSCCLPP_CUDATHROW(hipGetLastError());
  MSCCLPP_CUDATHROW(hipEventRecord(end, s1));
  MSCCLPP_CUDATHROW(hipEventSynchronize(end));
  float ms = 0;
  MSCCLPP_CUDATHROW(hipEventElapsedTime(&ms, start, end));
  MSCCLPP_CUDATHROW(hipSetDevice(dev0));
  MSCCLPP_CUDATHROW(hipStreamSynchronize(s0));
  // every signal landed: each side's token counts the other's iter signals
  uint64_t tok0 = 0, tok1 = 0;
  MSCCLPP_CUDATHROW(hipMemcpy(&tok0, sema0.localMemory().data(), 8, hipMemcpyDeviceToHost));
  MSCCLPP_CUDATHROW(hipMemcpy(&tok1, sema1.localMemory().data(), 8, hipMemcpyDeviceToHost));
  const float perIter = ms / iter;
  std::printf("context: %d rounds, %.3f ms per round, tokens %llu %llu (GPUs %d, %d)\n", iter, perIter,
              (unsigned long long)tok0, (unsigned long long)tok1, dev0, dev1);
  CHECK(tok0 == (uint64_t)iter && tok1 == (uint64_t)iter);
  CHECK(perIter >= 0.09f);  // each round waited for the other side's 100 us spin
  std::printf("context OK\n");
  return 0;
}

// ---- port: the port-channel tutorial ----------------------------------------------------------------
__global__ void bidirPortPutKernel(mscclpp::PortChannelDeviceHandle* h, size_t copyBytes, int myRank) {
  if (threadIdx.x + blockIdx.x * blockDim.x == 0) {
    h->signal();
    h->wait();
    const uint64_t off = myRank * copyBytes;
    h->putWithSignal(off, off, copyBytes);
    h->wait();
  }
}

static int portWorker(int myRank, const std::string& ipPort) {
  MSCCLPP_CUDATHROW(hipSetDevice(0));
  int gpuId = 0;
  MSCCLPP_CUDATHROW(hipGetDevice(&gpuId));
  // the tutorial's shape: 1000 graph-captured iterations of 1 KiB, 1 MiB and 128 MiB
  // (bidir_port_channel.cu:70-75, :119-170)
  const int remoteRank = myRank ^ 1, nRanks = 2, iter = 1000;
  const mscclpp::Transport transport = mscclpp::Transport::CudaIpc;
  const size_t maxBytes = (size_t)128 << 20;
  auto bootstrap = std::make_shared<mscclpp::TcpBootstrap>(myRank, nRanks);
  bootstrap->initialize(ipPort);
  mscclpp::Communicator comm(bootstrap);
  auto conn = comm.connect({transport, {mscclpp::DeviceType::GPU, gpuId}}, remoteRank).get();
  auto sema = comm.buildSemaphore(conn, remoteRank).get();
  mscclpp::GpuBuffer buffer(2 * maxBytes);
  auto localRegMem = comm.registerMemory(buffer.data(), buffer.bytes(), transport);
  comm.sendMemory(localRegMem, remoteRank);
  auto remoteRegMem = comm.recvMemory(remoteRank).get();

  mscclpp::ProxyService proxyService;
  mscclpp::SemaphoreId semaId = proxyService.addSemaphore(sema);
  mscclpp::MemoryId localMemId = proxyService.addMemory(localRegMem);
  mscclpp::MemoryId remoteMemId = proxyService.addMemory(remoteRegMem);
  mscclpp::PortChannel portChan = proxyService.portChannel(semaId, remoteMemId, localMemId);
  auto handle = portChan.deviceHandle();
  auto dev = mscclpp::detail::gpuCallocShared<mscclpp::PortChannelDeviceHandle>();
  mscclpp::gpuMemcpy(dev.get(), &handle, 1, hipMemcpyHostToDevice);
  hipStream_t stream;
  MSCCLPP_CUDATHROW(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  int* buf = (int*)buffer.data();
  int round = 0;
  for (size_t copyBytes : {(size_t)1024, (size_t)1 << 20, maxBytes}) {
    const size_t n = copyBytes / sizeof(int);
    auto mine = pattern(myRank, n, 20 + round);
    mscclpp::gpuMemcpy(buf + myRank * n, mine.data(), n, hipMemcpyHostToDevice);  // at myRank * copyBytes
    MSCCLPP_CUDATHROW(hipDeviceSynchronize());
    // the tutorial's sequence: capture with the proxy stopped, replay with it running
    proxyService.startProxy();
    hipGraph_t graph;
    hipGraphExec_t graphExec;
    MSCCLPP_CUDATHROW(hipStreamBeginCapture(stream, hipStreamCaptureModeGlobal));
    for (int i = 0; i < iter; ++i)
      hipLaunchKernelGGL(bidirPortPutKernel, dim3(1), dim3(1), 0, stream, dev.get(), copyBytes, myRank);
    MSCCLPP_CUDATHROW(hipStreamEndCapture(stream, &graph));
    MSCCLPP_CUDATHROW(hipGraphInstantiate(&graphExec, graph, nullptr, nullptr, 0));
    proxyService.stopProxy();
    MSCCLPP_CUDATHROW(hipDeviceSynchronize());
    proxyService.startProxy();
    bootstrap->barrier();
    hipEvent_t start, end;
    MSCCLPP_CUDATHROW(hipEventCreate(&start));
    MSCCLPP_CUDATHROW(hipEventCreate(&end));
    MSCCLPP_CUDATHROW(hipEventRecord(start, stream));
    MSCCLPP_CUDATHROW(hipGraphLaunch(graphExec, stream));
    MSCCLPP_CUDATHROW(hipEventRecord(end, stream));
    MSCCLPP_CUDATHROW(hipStreamSynchronize(stream));
    uint32_t rec[4] = {0, 0, 0, 0};
    MSCCLPP_CUDATHROW(hipMemcpy(rec, comm.deviceErrorWord(), sizeof(rec), hipMemcpyDeviceToHost));
    if (rec[0]) {
      std::printf("rank %d [Bidir PutWithSignal] bytes %zu: device error %u (%u, %u, %u)\n", myRank, copyBytes, rec[0],
                  rec[1], rec[2], rec[3]);
      std::fflush(stdout);
    }
    CHECK(rec[0] == 0);
    if (myRank == 0) {  // the tutorial's line (bidir_port_channel.cu:155-161)
      float ms = 0;
      MSCCLPP_CUDATHROW(hipEventElapsedTime(&ms, start, end));
      const float perIter = ms / iter;
      std::printf("Rank %d: [Bidir PutWithSignal] bytes %zu, elapsed %g ms/iter, BW %g GB/s\n", myRank, copyBytes,
                  perIter, (float)copyBytes / perIter * 1e-6f);
      std::printf("PORT_JSON {\"bytes\": %zu, \"us_per_iter\": %.3f, \"GBs\": %.3f, \"iters\": %d}\n", copyBytes,
                  perIter * 1e3, (float)copyBytes / perIter * 1e-6f, iter);
      std::fflush(stdout);
    }
    MSCCLPP_CUDATHROW(hipEventDestroy(start));
    MSCCLPP_CUDATHROW(hipEventDestroy(end));
    proxyService.stopProxy();
    bootstrap->barrier();
    std::vector<int> got(n);
    mscclpp::gpuMemcpy(got.data(), buf + remoteRank * n, n, hipMemcpyDeviceToHost);
    const auto want = pattern(remoteRank, n, 20 + round);
    size_t bad = 0;
    for (size_t i = 0; i < n; ++i) bad += got[i] != want[i];
    if (bad) std::fprintf(stderr, "rank %d port %zu bytes: %zu of %zu words wrong\n", myRank, copyBytes, bad, n);
    CHECK(bad == 0);
    MSCCLPP_CUDATHROW(hipGraphExecDestroy(graphExec));
    MSCCLPP_CUDATHROW(hipGraphDestroy(graph));
    ++round;
  }
  MSCCLPP_CUDATHROW(hipStreamDestroy(stream));
  bootstrap->barrier();
  std::printf("rank %d port OK\n", myRank);
  std::fflush(stdout);
  return 0;
}

// ---- executor: the reference's executor_test sequence -------------------------------------------
static int executorWorker(int rank, mscclpp::UniqueId id, const std::string& planPath) {
  MSCCLPP_CUDATHROW(hipSetDevice(0));
  const int worldSize = 2;
  auto bootstrap = std::make_shared<mscclpp::TcpBootstrap>(rank, worldSize);
  bootstrap->initialize(id);
  auto communicator = std::make_shared<mscclpp::Communicator>(bootstrap);
  auto executor = std::make_shared<mscclpp::Executor>(communicator);
  mscclpp::ExecutionPlan plan(planPath, rank);
  CHECK(plan.collective() == "allreduce" && plan.isInPlace());
  const size_t count = 1 << 16, bufferSize = count * sizeof(_Float16);
  std::shared_ptr<char> sendbuff = mscclpp::GpuBuffer(bufferSize).memory();
  hipStream_t stream;
  MSCCLPP_CUDATHROW(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  std::vector<_Float16> h(count), got(count);
  int call = 0;
  for (mscclpp::PacketType pt : {mscclpp::PacketType::LL16, mscclpp::PacketType::LL8}) {
    for (int it = 0; it < 3; ++it, ++call) {
      // small integers: every partial sum is exact in fp16, so any reduction order gives the same bits
      for (size_t i = 0; i < count; ++i) h[i] = (_Float16)(float)((i * 7 + call * 3 + rank * 5) % 61);
      mscclpp::gpuMemcpy(sendbuff.get(), (const char*)h.data(), bufferSize, hipMemcpyHostToDevice);
      bootstrap->barrier();
      executor->execute(rank, sendbuff.get(), sendbuff.get(), bufferSize, bufferSize, mscclpp::DataType::FLOAT16, plan,
                        stream, pt);
      MSCCLPP_CUDATHROW(hipStreamSynchronize(stream));
      mscclpp::gpuMemcpy((char*)got.data(), sendbuff.get(), bufferSize, hipMemcpyDeviceToHost);
      size_t bad = 0;
      for (size_t i = 0; i < count; ++i) {
        float want = 0;
        for (int r = 0; r < worldSize; ++r) want += (float)((i * 7 + call * 3 + r * 5) % 61);
        bad += (float)got[i] != want;
      }
      if (bad) std::fprintf(stderr, "rank %d call %d: %zu of %zu wrong\n", rank, call, bad, count);
      CHECK(bad == 0);
      bootstrap->barrier();
    }
  }
  // a bad argument is an exception, as in the reference
  bool threw = false;
  try {
    executor->execute(rank, nullptr, nullptr, bufferSize, bufferSize, mscclpp::DataType::FLOAT16, plan, stream);
  } catch (const mscclpp::Error& e) {
    threw = e.getErrorCode() == mscclpp::ErrorCode::InvalidUsage;
  }
  CHECK(threw);
  MSCCLPP_CUDATHROW(hipStreamDestroy(stream));
  bootstrap->barrier();
  std::printf("rank %d executor OK\n", rank);
  std::fflush(stdout);
  return 0;
}

// Two ranks in forked children.  A rank that throws says where (its own line) and exits 1; the first
// rank to fail ends the other at once (SIGKILL), which would otherwise wait out the spin budget of
// every remaining launch of its captured graphs for a peer that is gone.
static int forkPair(const std::function<int(int)>& worker, const char* name) {
  std::vector<pid_t> pids;
  for (int r = 0; r < 2; ++r) {
    const pid_t pid = fork();
    CHECK(pid >= 0);
    if (pid == 0) {
      int rc = 1;
      try {
        rc = worker(r);
      } catch (const std::exception& e) {
        std::printf("rank %d %s threw: %s\n", r, name, e.what());
      }
      std::fflush(stdout);
      std::_Exit(rc);
    }
    pids.push_back(pid);
  }
  int bad = 0, left = 2;
  while (left > 0) {
    int st = 0;
    const pid_t pid = waitpid(-1, &st, 0);
    if (pid < 0) break;
    const int r = pid == pids[0] ? 0 : pid == pids[1] ? 1 : -1;
    if (r < 0) continue;
    --left;
    if (WIFEXITED(st) && WEXITSTATUS(st) == 0) continue;
    ++bad;
    std::printf("rank %d %s ended with %s %d\n", r, name, WIFEXITED(st) ? "exit status" : "signal",
                WIFEXITED(st) ? WEXITSTATUS(st) : WTERMSIG(st));
    if (left > 0) {
      std::printf("rank %d %s: stopping rank %d\n", r, name, 1 - r);
      (void)kill(pids[1 - r], SIGKILL);
    }
    std::fflush(stdout);
  }
  std::printf(bad ? "%s FAILED\n" : "%s OK\n", name);
  return bad ? 1 : 0;
}

// test/unit/numa_tests.cc, utils_tests.cc and errors: host utilities as the reference's unit tests
// call them, plus one kernel on the atomic / poll spellings (a producer block publishes with
// atomicStore release, a consumer block waits with POLL_MAYBE_JAILBREAK on atomicLoad acquire).
__global__ void kernelAtomicPoll(int* data, uint32_t* flag, int* out) {
  if (blockIdx.x == 0) {
    if (threadIdx.x == 0) {
      data[0] = 42;
      mscclpp::atomicStore<uint32_t, mscclpp::scopeDevice>(flag, 1u, mscclpp::memoryOrderRelease);
    }
  } else if (threadIdx.x == 0) {
    POLL_MAYBE_JAILBREAK((mscclpp::atomicLoad<uint32_t, mscclpp::scopeDevice>(flag, mscclpp::memoryOrderAcquire) == 0),
                         -1);
    out[0] = data[0];
    (void)mscclpp::atomicFetchAdd<uint32_t, mscclpp::scopeDevice>(flag, 1u, mscclpp::memoryOrderRelaxed);
  }
}

static int runUtils() {
  int num = 0;
  MSCCLPP_CUDATHROW(hipGetDeviceCount(&num));
  for (int i = 0; i < num; i++) {
    const int node = mscclpp::getDeviceNumaNode(i);
    CHECK(node >= -1);  // a container without the PCI sysfs entry reports -1
    if (node >= 0) mscclpp::numaBind(node);
  }
  const std::string h1 = mscclpp::getHostName(1024, '.');
  CHECK(!h1.empty() && h1.size() <= 1024);
  CHECK(mscclpp::getHostName(1024, h1[0]).empty());
  CHECK(mscclpp::env()->logLevel.size() > 0 && mscclpp::env() == mscclpp::env());
  bool threw = false;
  try {
    MSCCLPP_CUDATHROW(hipSetDevice(1 << 20));
  } catch (const mscclpp::CudaError& e) {
    threw = e.getErrorCode() != 0 && std::string(e.what()).find("Cuda failure") != std::string::npos;
  }
  CHECK(threw);
  (void)hipGetLastError();  // clear the invalid-device error the check above provoked
  try {
    throw mscclpp::Error("x", mscclpp::ErrorCode::Timeout);
  } catch (const mscclpp::BaseError& e) {
    CHECK(e.getErrorCode() == (int)mscclpp::ErrorCode::Timeout);
    CHECK(std::string(e.what()) == "x (mscclpp failure: Timeout)");
  }
  auto data = mscclpp::detail::gpuCallocShared<int>(1);
  auto flag = mscclpp::detail::gpuCallocShared<uint32_t>(1);
  auto out = mscclpp::detail::gpuCallocShared<int>(1);
  hipLaunchKernelGGL(kernelAtomicPoll, dim3(2), dim3(64), 0, 0, data.get(), flag.get(), out.get());
  MSCCLPP_CUDATHROW(hipGetLastError());
  MSCCLPP_CUDATHROW(hipDeviceSynchronize());
  int o = 0;
  uint32_t f = 0;
  MSCCLPP_CUDATHROW(hipMemcpy(&o, out.get(), sizeof(o), hipMemcpyDeviceToHost));
  MSCCLPP_CUDATHROW(hipMemcpy(&f, flag.get(), sizeof(f), hipMemcpyDeviceToHost));
  CHECK(o == 42 && f == 2);
  std::printf("utils OK\n");
  return 0;
}

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "";
  if (mode == "utils") return runUtils();
  if (mode == "local") return runLocal();
  if (mode == "context") return runContext();
  if (mode == "pair" && argc > 2) {
    const std::string ipPort = std::string("127.0.0.1:") + argv[2];
    return forkPair([&](int r) { return pairWorker(r, ipPort); }, "pair");
  }
  if (mode == "uid") {
    // the id is created here, before any child touches the GPU (the root thread lives in this
    // process); no HIP call is made in the parent
    const mscclpp::UniqueId id = mscclpp::TcpBootstrap::createUniqueId();
    return forkPair([&](int r) { return uidWorker(r, id); }, "uid");
  }
  if (mode == "port" && argc > 2) {
    const std::string ipPort = std::string("127.0.0.1:") + argv[2];
    return forkPair([&](int r) { return portWorker(r, ipPort); }, "port");
  }
  if (mode == "executor" && argc > 2) {
    const std::string planPath = argv[2];
    const mscclpp::UniqueId id = mscclpp::TcpBootstrap::createUniqueId();
    return forkPair([&](int r) { return executorWorker(r, id, planPath); }, "executor");
  }
  std::fprintf(stderr, "usage: %s local | pair PORT | uid | context | port PORT | executor PLAN\n", argv[0]);
  return 2;
}
