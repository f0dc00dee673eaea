// Two ranks (processes), channels built with the host API (core.hpp, semaphore.hpp,
// memory_channel.hpp, port_channel.hpp) exactly as a user of the reference builds them, driven by
// kernels written with the reference's device spellings.  Everything is included through the
// reference's paths (include/mscclpp/*.hpp, forwarding to include/mscclpp_amd) and spelled
// mscclpp::..., with no alias or rename; only the harness's C entry points come
// from mscclpp_amd.h:
//   memory channel  LL8 / LL16 packet ping-pong     test/mp_unit/memory_channel_tests.cu:246-325
//                   put + signal / wait ping-pong    memory_channel_tests.cu (put ping-pong)
//                   get ping-pong                    memory_channel_tests.cu (get ping-pong)
//                   unpackPacket(index, flag)        memory_channel_device.hpp:178-182
//   port channel    proxy LL ping-pong: copyToPackets -> put -> copyFromPackets, flush every 64
//                   (test/mp_unit/port_channel_tests.cu:337-446)
//                   putWithSignal / wait ping-pong    port_channel_tests.cu (ping-pong)
//
//   test_channels gpu [nElemMax]   forks 2 ranks (rank % device count)
#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <type_traits>
#include <vector>

#include <mscclpp/core.hpp>
#include <mscclpp/ext/nccl/nccl.h>
#include <mscclpp/gpu_utils.hpp>
#include <mscclpp/memory_channel.hpp>
#include <mscclpp/memory_channel_device.hpp>
#include <mscclpp/packet_device.hpp>
#include <mscclpp/port_channel.hpp>
#include <mscclpp/port_channel_device.hpp>

#include "mscclpp_amd/mscclpp_amd.h"

using mscclpp::DeviceHandle;

#define CHECK(cond)                                                                              \
  do {                                                                                           \
    if (!(cond)) {                                                                               \
      std::fprintf(stderr, "[rank %d] CHECK failed %s:%d: %s\n", gRank, __FILE__, __LINE__, #cond); \
      std::exit(1);                                                                              \
    }                                                                                            \
  } while (0)
#define HIP_OK(cmd) CHECK((cmd) == hipSuccess)

static int gRank = -1;

// Flag ranges of the packet ping-pongs.  Each (size, packet type) case and the timed run get a range
// of their own, so a packet slot never holds a flag a later case waits for: no clear of the packet
// buffer is needed between cases (the reference's packetPingPongTest does not clear either,
// memory_channel_tests.cu:91-96).
constexpr uint32_t kCaseFlagStride = 1u << 12;      // >= nTries of a correctness case (1000)
constexpr uint32_t kTimedFlagBase = 1u << 20;       // the timed ping-pongs: up to 2^20 tries each
constexpr uint32_t kUnpackFlagBase = 3u << 21;      // unpackPacket: beyond both timed ranges
constexpr int kTimedTries = 100000;                 // timed ping-pong iterations (>= 100k)

__constant__ DeviceHandle<mscclpp::MemoryChannel> gChannelOneToOneTestConstMemChans;
__constant__ DeviceHandle<mscclpp::PortChannel> gChannelOneToOneTestConstPortChans;

// ---- memory channel ---------------------------------------------------------------------------
__global__ void kernelMemLL8PacketPingPong(int* buff, int rank, int nElem, int* ret, int nTries, uint32_t flagBase) {
  if (rank > 1) return;
  DeviceHandle<mscclpp::MemoryChannel>& memChan = gChannelOneToOneTestConstMemChans;
  volatile int* sendBuff = (volatile int*)buff;
  int putOffset = (rank == 0) ? 0 : 10000000;
  int getOffset = (rank == 0) ? 10000000 : 0;
  for (int i = 0; i < nTries; i++) {
    uint64_t flag = (uint64_t)flagBase + i + 1;
    if ((rank ^ (i & 1)) == 0) {
      for (int j = threadIdx.x; j < nElem; j += blockDim.x) sendBuff[j] = putOffset + i + j;
      memChan.putPackets<mscclpp::LL8Packet>(0, 0, nElem * sizeof(int), threadIdx.x, blockDim.x, flag);
    } else {
      memChan.unpackPackets<mscclpp::LL8Packet>(0, 0, nElem * sizeof(int), threadIdx.x, blockDim.x, flag);
      for (int j = threadIdx.x; j < nElem; j += blockDim.x) {
        if (sendBuff[j] != getOffset + i + j) {
          *ret = 1;
          break;
        }
      }
    }
    __syncthreads();
  }
}

__global__ void kernelMemLL16PacketPingPong(int* buff, int rank, int nElem, int* ret, int nTries, uint32_t flagBase) {
  if (rank > 1) return;
  DeviceHandle<mscclpp::MemoryChannel>& memChan = gChannelOneToOneTestConstMemChans;
  volatile int* sendBuff = (volatile int*)buff;
  int putOffset = (rank == 0) ? 0 : 10000000;
  int getOffset = (rank == 0) ? 10000000 : 0;
  for (int i = 0; i < nTries; i++) {
    uint64_t flag = (uint64_t)flagBase + i + 1;
    if ((rank ^ (i & 1)) == 0) {
      for (int j = threadIdx.x; j < nElem / 2; j += blockDim.x) {
        sendBuff[2 * j] = putOffset + i + 2 * j;
        sendBuff[2 * j + 1] = putOffset + i + 2 * j + 1;
      }
      memChan.putPackets<mscclpp::LL16Packet>(0, 0, nElem * sizeof(int), threadIdx.x, blockDim.x, flag);
    } else {
      memChan.unpackPackets<mscclpp::LL16Packet>(0, 0, nElem * sizeof(int), threadIdx.x, blockDim.x, flag);
      for (int j = threadIdx.x; j < nElem / 2; j += blockDim.x) {
        if (sendBuff[2 * j] != getOffset + i + 2 * j || sendBuff[2 * j + 1] != getOffset + i + 2 * j + 1) {
          *ret = 1;
          break;
        }
      }
    }
    __syncthreads();
  }
}

// unpackPacket(index, flag): each thread reads single packets of the local packet buffer
__global__ void kernelMemUnpackPacket(int* buff, int rank, int nElem, int* ret, int nTries) {
  DeviceHandle<mscclpp::MemoryChannel>& memChan = gChannelOneToOneTestConstMemChans;
  volatile int* sendBuff = (volatile int*)buff;
  int putOffset = (rank == 0) ? 0 : 10000000;
  int getOffset = (rank == 0) ? 10000000 : 0;
  for (int i = 0; i < nTries; i++) {
    uint32_t flag = (uint32_t)(kUnpackFlagBase + i);  // beyond every flag the ping-pongs above used
    if ((rank ^ (i & 1)) == 0) {
      for (int j = threadIdx.x; j < nElem; j += blockDim.x) sendBuff[j] = putOffset + i + 7 * j;
      memChan.putPackets(0, 0, nElem * sizeof(int), threadIdx.x, blockDim.x, flag);
    } else {
      for (int j = threadIdx.x; j < nElem / 2; j += blockDim.x) {
        uint2 v = memChan.unpackPacket(j, flag);
        if ((int)v.x != getOffset + i + 7 * (2 * j) || (int)v.y != getOffset + i + 7 * (2 * j + 1)) *ret = 1;
      }
      static_assert(std::is_same<decltype(memChan.unpackPacket<mscclpp::LL8Packet>(0, 0)), uint32_t>::value,
                    "unpackPacket<LL8Packet> returns the 4-byte payload");
      static_assert(std::is_same<decltype(memChan.unpackPacket(0, 0)), uint2>::value,
                    "unpackPacket<LL16Packet> returns the 8-byte payload");
    }
    __syncthreads();
  }
}

// put + signal / wait, then read back what the peer put (memory_channel_tests.cu put ping-pong)
__global__ void kernelMemPutPingPong(int* buff, int rank, int nElem, int* ret, int nTries) {
  DeviceHandle<mscclpp::MemoryChannel>& memChan = gChannelOneToOneTestConstMemChans;
  volatile int* sendBuff = (volatile int*)buff;
  const int half = nElem / 2;
  for (int i = 0; i < nTries; i++) {
    // my half of my buffer -> the same half of the peer's buffer
    for (int j = threadIdx.x; j < half; j += blockDim.x) sendBuff[rank * half + j] = rank * 1000000 + i + j;
    __syncthreads();
    memChan.put<16, true>(rank * half * sizeof(int), half * sizeof(int), threadIdx.x, blockDim.x);
    __syncthreads();
    if (threadIdx.x == 0) {
      memChan.signal();
      memChan.wait();
    }
    __syncthreads();
    const int peer = 1 - rank;
    for (int j = threadIdx.x; j < half; j += blockDim.x)
      if (sendBuff[peer * half + j] != peer * 1000000 + i + j) *ret = 1;
    __syncthreads();
    if (threadIdx.x == 0) {  // both are done reading before the next round's puts
      memChan.relaxedSignal();
      memChan.relaxedWait();
    }
    __syncthreads();
  }
}

// get: read the peer's own half straight out of its buffer
__global__ void kernelMemGetPingPong(int* buff, int rank, int nElem, int* ret, int nTries) {
  DeviceHandle<mscclpp::MemoryChannel>& memChan = gChannelOneToOneTestConstMemChans;
  volatile int* sendBuff = (volatile int*)buff;
  const int half = nElem / 2;
  const int peer = 1 - rank;
  for (int i = 0; i < nTries; i++) {
    for (int j = threadIdx.x; j < half; j += blockDim.x) sendBuff[rank * half + j] = rank * 3000000 + 5 * i + j;
    __syncthreads();
    if (threadIdx.x == 0) {
      memChan.signal();
      memChan.wait();
    }
    __syncthreads();
    memChan.get(peer * half * sizeof(int), half * sizeof(int), threadIdx.x, blockDim.x);
    __syncthreads();
    for (int j = threadIdx.x; j < half; j += blockDim.x)
      if (sendBuff[peer * half + j] != peer * 3000000 + 5 * i + j) *ret = 1;
    __syncthreads();
    if (threadIdx.x == 0) {
      memChan.signal();
      memChan.wait();
    }
    __syncthreads();
  }
}

// ---- port channel ------------------------------------------------------------------------------
__global__ void kernelProxyLLPingPong(int* buff, mscclpp::LLPacket* putPktBuf, mscclpp::LLPacket* getPktBuf, int rank,
                                      int nElem, int nTries, int* ret) {
  if (rank > 1) return;
  DeviceHandle<mscclpp::PortChannel>& portChan = gChannelOneToOneTestConstPortChans;
  volatile int* buffPtr = (volatile int*)buff;
  int putOffset = (rank == 0) ? 0 : 10000000;
  int getOffset = (rank == 0) ? 10000000 : 0;
  int threadId = threadIdx.x + blockIdx.x * blockDim.x;
  int numThreads = blockDim.x * gridDim.x;
  int flusher = 0;
  const int nPkt = nElem / 2;
  for (int i = 0; i < nTries; i++) {
    uint64_t flag = (uint64_t)i + 1;
    if ((rank ^ (i & 1)) == 0) {
      for (int j = threadId; j < nPkt; j += numThreads) {
        buffPtr[2 * j] = putOffset + i + 2 * j;
        buffPtr[2 * j + 1] = putOffset + i + 2 * j + 1;
      }
      mscclpp::copyToPackets(putPktBuf, buff, nElem * sizeof(int), threadId, numThreads, flag);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadId == 0) portChan.put(0, nPkt * sizeof(mscclpp::LLPacket));
      flusher++;
      if (flusher == 64) {
        if (threadId == 0) portChan.flush();
        flusher = 0;
      }
    } else {
      mscclpp::copyFromPackets(buff, getPktBuf, nElem * sizeof(int), threadId, numThreads, flag);
      for (int j = threadId; j < nPkt; j += numThreads) {
        if (buffPtr[2 * j] != getOffset + i + 2 * j || buffPtr[2 * j + 1] != getOffset + i + 2 * j + 1) {
          *ret = 1;
          break;
        }
      }
      __syncthreads();
    }
  }
  if (threadId == 0) portChan.flush();
}

// putWithSignal + wait: my half -> the peer's buffer, then check the peer's half arrived in mine
__global__ void kernelPortPutPingPong(int* buff, int rank, int nElem, int* ret, int nTries) {
  DeviceHandle<mscclpp::PortChannel>& portChan = gChannelOneToOneTestConstPortChans;
  volatile int* p = (volatile int*)buff;
  const int half = nElem / 2;
  const int peer = 1 - rank;
  for (int i = 0; i < nTries; i++) {
    for (int j = threadIdx.x; j < half; j += blockDim.x) p[rank * half + j] = rank * 2000000 + 3 * i + j;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      if (i % 2)
        portChan.putWithSignal(rank * half * sizeof(int), half * sizeof(int));
      else
        portChan.putWithSignalAndFlush(rank * half * sizeof(int), half * sizeof(int));
      portChan.wait();
    }
    __syncthreads();
    for (int j = threadIdx.x; j < half; j += blockDim.x)
      if (p[peer * half + j] != peer * 2000000 + 3 * i + j) *ret = 1;
    __syncthreads();
    if (threadIdx.x == 0) {  // both have read before the next round overwrites
      portChan.signal();
      portChan.flush();
      portChan.wait();
    }
    __syncthreads();
  }
}

// A trigger carries 32-bit offsets and size (fifo_device.hpp:71-77): oversize puts are refused on the
// device -- nothing pushed, kErrBadGeometry in the error word -- instead of being truncated.
__global__ void kernelPortOversizePut() {
  if (threadIdx.x == 0) {
    DeviceHandle<mscclpp::PortChannel>& c = gChannelOneToOneTestConstPortChans;
    c.put(0, 0, 1ull << 32);
    c.putWithSignal(1ull << 32, 0, 16);
    c.putWithSignalAndFlush(0, 1ull << 32, 16);
  }
}

static int worker(int rank, ncclUniqueId id, int nElemMax) {
  gRank = rank;
  int ndev = 0;
  HIP_OK(hipGetDeviceCount(&ndev));
  HIP_OK(hipSetDevice(rank % ndev));
  auto comm = mscclpp::Communicator::create(rank, 2, id);
  const int peer = 1 - rank;
  CHECK(comm->bootstrap()->getRank() == rank && comm->bootstrap()->getNranks() == 2);
  CHECK(comm->bootstrap()->getNranksPerNode() == 2);

  // bootstrap point-to-point: tags are matched independently, in order per (peer, tag)
  {
    int a = rank * 10 + 1, b = rank * 10 + 2, x = -1, y = -1;
    comm->bootstrap()->send(&b, sizeof(b), peer, 7);
    comm->bootstrap()->send(&a, sizeof(a), peer, 3);
    comm->bootstrap()->recv(&x, sizeof(x), peer, 3);
    comm->bootstrap()->recv(&y, sizeof(y), peer, 7);
    CHECK(x == peer * 10 + 1 && y == peer * 10 + 2);
    int all[2] = {0, 0};
    all[rank] = 40 + rank;
    comm->bootstrap()->allGather(all, sizeof(int));
    CHECK(all[0] == 40 && all[1] == 41);
  }

  const size_t bytes = (size_t)nElemMax * sizeof(int);
  // uncached, as the reference test's mscclpp::GpuBuffer is on AMD (gpu_utils.hpp:375-376)
  auto buff = mscclpp::detail::gpuCallocUncachedShared<int>(nElemMax);
  auto pkt = mscclpp::detail::gpuCallocUncachedShared<mscclpp::LL16Packet>(nElemMax);  // LL8 needs nElem, LL16 nElem/2
  auto putPkt = mscclpp::detail::gpuCallocUncachedShared<mscclpp::LLPacket>(nElemMax / 2 + 1);
  auto getPkt = mscclpp::detail::gpuCallocUncachedShared<mscclpp::LLPacket>(nElemMax / 2 + 1);
  auto ret = mscclpp::detail::gpuCallocShared<int>(1);

  auto connF = comm->connect(mscclpp::Transport::CudaIpc, peer);
  mscclpp::RegisteredMemory buffMem = comm->registerMemory(buff.get(), bytes, mscclpp::Transport::CudaIpc);
  mscclpp::RegisteredMemory pktMem = comm->registerMemory(pkt.get(), bytes * 2, mscclpp::Transport::CudaIpc);
  const size_t pktBytes = (nElemMax / 2 + 1) * sizeof(mscclpp::LLPacket);
  mscclpp::RegisteredMemory putPktMem = comm->registerMemory(putPkt.get(), pktBytes, mscclpp::Transport::CudaIpc);
  mscclpp::RegisteredMemory getPktMem = comm->registerMemory(getPkt.get(), pktBytes, mscclpp::Transport::CudaIpc);
  comm->sendMemory(buffMem, peer, 0);
  comm->sendMemory(pktMem, peer, 1);
  comm->sendMemory(getPktMem, peer, 2);
  auto remoteBuffF = comm->recvMemory(peer, 0);
  auto remotePktF = comm->recvMemory(peer, 1);
  auto remoteGetPktF = comm->recvMemory(peer, 2);
  mscclpp::Connection conn = connF.get();
  CHECK(comm->remoteRankOf(conn) == peer && comm->tagOf(conn) == 0);
  CHECK(conn.transport() == mscclpp::Transport::CudaIpc);
  mscclpp::RegisteredMemory remoteBuff = remoteBuffF.get(), remotePkt = remotePktF.get();
  mscclpp::RegisteredMemory remoteGetPkt = remoteGetPktF.get();
  CHECK(remoteBuff.size() == bytes && remoteBuff.rank() == peer && remoteBuff.data() != nullptr);
  // serialize / deserialize round trip of a local registration stays local
  {
    auto again = mscclpp::RegisteredMemory::deserialize(buffMem.serialize());
    CHECK(again.data() == buff.get() && again.size() == bytes);
  }

  auto sem = std::make_shared<mscclpp::MemoryDevice2DeviceSemaphore>(*comm, conn);
  int* r = ret.get();
  // A failed case prints the error record: for a packet timeout the flag waited for, the packet's
  // byte offset and the flag word last read there (mscclppAmdCommGetDeviceErrorDetail).
  auto verdict = [&](const char* name, int nElem, int h) {
    uint32_t w[4] = {0, 0, 0, 0};
    CHECK(mscclppAmdCommGetDeviceErrorDetail(comm->ncclComm(), w, 1) == 0);
    if (h != 0 || w[0] != 0) {
      std::fprintf(stderr, "[rank %d] %s nElem %d: ret %d device error %u (flag %u, packet byte %u, flag seen %u)\n",
                   rank, name, nElem, h, w[0], w[1], w[2], w[3]);
      std::exit(1);
    }
  };
  // Every host-side fill (hipMemset of the result word) has completed on the device before the
  // barrier that lets the peer launch: a fill still queued behind the barrier could land after the
  // peer's first stores.
  auto launch = [&](auto&& go) {
    HIP_OK(hipMemset(r, 0, sizeof(int)));
    HIP_OK(hipDeviceSynchronize());
    comm->bootstrap()->barrier();
    go();
    HIP_OK(hipGetLastError());
    HIP_OK(hipDeviceSynchronize());
    int h = -1;
    HIP_OK(hipMemcpy(&h, r, sizeof(int), hipMemcpyDeviceToHost));
    return h;
  };
  auto run = [&](const char* name, auto kernel, int nElem, int nTries) {
    const int h = launch([&] { hipLaunchKernelGGL(kernel, dim3(1), dim3(1024), 0, 0, buff.get(), rank, nElem, r, nTries); });
    verdict(name, nElem, h);
    comm->bootstrap()->barrier();
  };
  auto runPkt = [&](const char* name, auto kernel, int nElem, int nTries, uint32_t flagBase) {
    const int h = launch(
        [&] { hipLaunchKernelGGL(kernel, dim3(1), dim3(1024), 0, 0, buff.get(), rank, nElem, r, nTries, flagBase); });
    verdict(name, nElem, h);
    comm->bootstrap()->barrier();
  };
  {
    // packet channel: my buff -> packets into the peer's packet buffer; mine receives
    mscclpp::MemoryChannel memChan(sem, remotePkt, buffMem, pkt.get());
    DeviceHandle<mscclpp::MemoryChannel> h = mscclpp::deviceHandle(memChan);
    HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(gChannelOneToOneTestConstMemChans), &h, sizeof(h)));
    // correctness: 1000 tries per size and packet type, each case in a flag range of its own
    // (memory_channel_tests.cu:91-96; the packet buffer is zeroed once, at allocation)
    uint32_t flagBase = 0;
    for (int n : {2, 1024, 1024 * 1024}) {
      if (n > nElemMax) continue;
      runPkt("LL8 ping-pong", kernelMemLL8PacketPingPong, n, 1000, flagBase);
      flagBase += kCaseFlagStride;
      runPkt("LL16 ping-pong", kernelMemLL16PacketPingPong, n, 1000, flagBase);
      flagBase += kCaseFlagStride;
    }
    CHECK(flagBase < kTimedFlagBase);
    // timed: kTimedTries one-way hand-offs of 1024 ints, the reference's latency measurement
    // (memory_channel_tests.cu:98-107: host timer between barriers around one launch, us/iter)
    if (nElemMax >= 1024) {
      const char* names[2] = {"LL8 ping-pong (timed)", "LL16 ping-pong (timed)"};
      double usPerIter[2] = {0, 0};
      for (int k = 0; k < 2; ++k) {
        HIP_OK(hipMemset(r, 0, sizeof(int)));
        HIP_OK(hipDeviceSynchronize());
        comm->bootstrap()->barrier();
        const auto t0 = std::chrono::steady_clock::now();
        if (k == 0)
          hipLaunchKernelGGL(kernelMemLL8PacketPingPong, dim3(1), dim3(1024), 0, 0, buff.get(), rank, 1024, r,
                             kTimedTries, kTimedFlagBase);
        else
          hipLaunchKernelGGL(kernelMemLL16PacketPingPong, dim3(1), dim3(1024), 0, 0, buff.get(), rank, 1024, r,
                             kTimedTries, kTimedFlagBase + (1u << 20));
        HIP_OK(hipGetLastError());
        HIP_OK(hipDeviceSynchronize());
        comm->bootstrap()->barrier();
        usPerIter[k] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() /
                       kTimedTries;
        int h = -1;
        HIP_OK(hipMemcpy(&h, r, sizeof(int), hipMemcpyDeviceToHost));
        verdict(names[k], 1024, h);
      }
      if (rank == 0)  // framework.cc:339-345's [   PERF   ] lines
        std::printf("[   PERF   ] MemoryChannelOneToOneTest.PacketPingPong\n"
                    "[   PERF   ]        LL8 latency: %.4g us/iter\n"
                    "[   PERF   ]       LL16 latency: %.4g us/iter\n"
                    "PINGPONG_JSON {\"ll8_pingpong_us\": %.4f, \"ll16_pingpong_us\": %.4f, \"nElem\": 1024, "
                    "\"iters\": %d}\n",
                    usPerIter[0], usPerIter[1], usPerIter[0], usPerIter[1], kTimedTries);
    }
    run("unpackPacket", kernelMemUnpackPacket, 4096, 50);
  }
  {
    // data channel: my buff -> the peer's buff
    mscclpp::MemoryChannel memChan(sem, remoteBuff, buffMem);
    DeviceHandle<mscclpp::MemoryChannel> h = memChan.deviceHandle();
    HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(gChannelOneToOneTestConstMemChans), &h, sizeof(h)));
    for (int n : {2, 1024 + 6, 1024 * 1024})
      if (n <= nElemMax) run("put ping-pong", kernelMemPutPingPong, n, 100);
    for (int n : {2, 1024 + 6, 1024 * 1024})
      if (n <= nElemMax) run("get ping-pong", kernelMemGetPingPong, n, 100);
  }
  {
    // port channels through the general ProxyService
    mscclpp::ProxyService proxy;
    const mscclpp::SemaphoreId sid = proxy.buildAndAddSemaphore(*comm, conn);
    const mscclpp::MemoryId putPktId = proxy.addMemory(putPktMem);
    const mscclpp::MemoryId remoteGetPktId = proxy.addMemory(remoteGetPkt);
    const mscclpp::MemoryId buffId = proxy.addMemory(buffMem);
    const mscclpp::MemoryId remoteBuffId = proxy.addMemory(remoteBuff);
    CHECK(proxy.nextMemoryId() == 4);
    proxy.startProxy();
    {
      DeviceHandle<mscclpp::PortChannel> h = mscclpp::deviceHandle(proxy.portChannel(sid, remoteGetPktId, putPktId));
      HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(gChannelOneToOneTestConstPortChans), &h, sizeof(h)));
      for (int n : {2, 1024, 1024 * 1024}) {
        if (n > nElemMax) continue;
        HIP_OK(hipMemset(getPkt.get(), 0, pktBytes));
        HIP_OK(hipMemset(r, 0, sizeof(int)));
        HIP_OK(hipDeviceSynchronize());  // both fills have landed before the peer may put into getPkt
        comm->bootstrap()->barrier();
        hipLaunchKernelGGL(kernelProxyLLPingPong, dim3(1), dim3(1024), 0, 0, buff.get(), putPkt.get(), getPkt.get(),
                           rank, n, 1000, r);
        HIP_OK(hipGetLastError());
        HIP_OK(hipDeviceSynchronize());
        int hr = -1;
        HIP_OK(hipMemcpy(&hr, r, sizeof(int), hipMemcpyDeviceToHost));
        verdict("proxy LL ping-pong", n, hr);
        comm->bootstrap()->barrier();
      }
    }
    {
      DeviceHandle<mscclpp::PortChannel> h = proxy.portChannel(sid, remoteBuffId, buffId).deviceHandle();
      HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(gChannelOneToOneTestConstPortChans), &h, sizeof(h)));
      for (int n : {2, 1024 + 6, 1024 * 1024})
        if (n <= nElemMax) run("port put ping-pong", kernelPortPutPingPong, n, 50);
      const uint64_t handled = proxy.triggersHandled();
      hipLaunchKernelGGL(kernelPortOversizePut, dim3(1), dim3(64), 0, 0);
      HIP_OK(hipGetLastError());
      HIP_OK(hipDeviceSynchronize());
      uint32_t code = 0;
      CHECK(mscclppAmdCommGetDeviceError(comm->ncclComm(), &code, 1) == 0);
      CHECK(code == 4 /* kErrBadGeometry */);
      CHECK(proxy.triggersHandled() == handled);
      comm->bootstrap()->barrier();
    }
    CHECK(proxy.triggersHandled() > 0);
    proxy.stopProxy();
  }
  comm->bootstrap()->barrier();
  std::printf("rank %d OK\n", rank);
  std::fflush(stdout);
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 2 && std::string(argv[1]) == "gpu") {
    const int nElemMax = argc >= 3 ? std::atoi(argv[2]) : 1024 * 1024;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return 1;  // the root listens in this parent; no GPU touched
    std::vector<pid_t> pids;
    for (int r = 0; r < 2; ++r) {
      pid_t pid = fork();
      if (pid < 0) return 1;
      if (pid == 0) std::_Exit(worker(r, id, nElemMax));
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
  std::fprintf(stderr, "usage: %s gpu [nElemMax]\n", argv[0]);
  return 2;
}
