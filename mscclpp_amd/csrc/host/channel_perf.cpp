// The MemoryChannel packet ping-pong latency of the reference's mp_unit test
// (test/mp_unit/memory_channel_tests.cu:98-107: after the correctness sizes, one launch of 1,000,000
// one-way LL hand-offs of 1024 ints between two ranks, host timer between barriers, reported as
// us/iter), built with the host channel API exactly as a user builds it: connect, registerMemory,
// sendMemory / recvMemory, MemoryDevice2DeviceSemaphore, MemoryChannel(sem, remote packet buffer,
// local buffer, local packet buffer).
#include <chrono>

#include "comm_internal.hpp"
#include "mscclpp_amd/memory_channel.hpp"

extern "C" int mscclppAmdLaunchMemChannelPingPong(const void* handle, int* buff, int rank, int nElem, int nTries,
                                                  uint32_t flagBase, int ll8, int* ret, void* stream);

using namespace mscclpp_amd;

extern "C" {

// Collective over a 2-rank communicator.  First 1000 checked tries (flags 1..1000), then `iters`
// timed tries (flags 1001..) of nElem ints, LL8 (ll8 != 0) or LL16 packets.  out[0] = us per
// iteration (host clock from the barrier before the launch to the barrier after it, as the
// reference), out[1] = 1 if every receive matched and no device error was recorded, out[2..5] = the
// error record (code, flag, packet byte, flag seen).
int mscclppAmdMemChannelPingPong(ncclComm_t comm, int nElem, int iters, int ll8, double* out, int outLen) {
  return guarded([&] {
    if (!comm || !out || outLen < 2 || nElem <= 0 || nElem % 2 || iters <= 0 || iters > (1 << 30))
      return (int)ncclInvalidArgument;
    if (comm->nranks != 2) return (int)ncclInvalidArgument;
    const int rank = comm->rank, peer = 1 - rank;
    const size_t bytes = (size_t)nElem * 4;
    // released on every exit, a throw from the setup or a launch included
    struct Resources {
      int* buff = nullptr;
      void* pkt = nullptr;
      int* ret = nullptr;
      hipStream_t st = nullptr;
      ~Resources() {
        if (st) (void)hipStreamDestroy(st);
        if (ret) (void)hipFree(ret);
        if (pkt) releaseUncached(pkt, nullptr);
        if (buff) releaseUncached(buff, nullptr);
      }
    } res;
    res.buff = (int*)allocUncached(bytes);  // GpuBuffer on AMD: uncached (gpu_utils.cc:139-147)
    res.pkt = allocUncached(bytes * 2);     // LL16: nElem / 2 16-byte packets; LL8: nElem 8-byte
    HIPCHECK(hipMalloc((void**)&res.ret, sizeof(int)));
    HIPCHECK(hipStreamCreateWithFlags(&res.st, hipStreamNonBlocking));
    int* const buff = res.buff;
    void* const pkt = res.pkt;
    int* const ret = res.ret;
    const hipStream_t st = res.st;
    memsetSync(ret, 0, sizeof(int));
    double us = 0;
    int bad = 0;
    uint32_t rec[4] = {0, 0, 0, 0};
    {
      Communicator cx(comm);
      auto connF = cx.connect(Transport::CudaIpc, peer);
      RegisteredMemory buffMem = cx.registerMemory(buff, bytes, Transport::CudaIpc);
      RegisteredMemory pktMem = cx.registerMemory(pkt, bytes * 2, Transport::CudaIpc);
      cx.sendMemory(pktMem, peer);
      auto remotePktF = cx.recvMemory(peer);
      auto sem = std::make_shared<MemoryDevice2DeviceSemaphore>(cx, connF.get());
      MemoryChannel ch(sem, remotePktF.get(), buffMem, pkt);
      const MemoryChannelDeviceHandle h = ch.deviceHandle();
      // the zero fills of the allocations have completed before the peer may put into `pkt`
      HIPCHECK(hipDeviceSynchronize());
      comm->boot->barrier();
      if (mscclppAmdLaunchMemChannelPingPong(&h, buff, rank, nElem, 1000, 0, ll8, ret, st))
        throw std::runtime_error("ping-pong launch");
      HIPCHECK(hipStreamSynchronize(st));
      comm->boot->barrier();
      const auto t0 = std::chrono::steady_clock::now();
      if (mscclppAmdLaunchMemChannelPingPong(&h, buff, rank, nElem, iters, 1000, ll8, ret, st))
        throw std::runtime_error("ping-pong launch");
      HIPCHECK(hipStreamSynchronize(st));
      comm->boot->barrier();
      us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / iters;
      HIPCHECK(hipMemcpy(&bad, ret, sizeof(int), hipMemcpyDeviceToHost));
      HIPCHECK(hipMemcpy(rec, comm->err, sizeof(rec), hipMemcpyDeviceToHost));
      comm->boot->barrier();  // the peer is done with my packet buffer before its mapping closes
    }
    out[0] = us;
    out[1] = (bad == 0 && rec[0] == 0) ? 1.0 : 0.0;
    for (int k = 0; k < 4 && 2 + k < outLen; ++k) out[2 + k] = (double)rec[k];
    if (bad || rec[0])
      warn("MemoryChannel ping-pong rank " + std::to_string(rank) + ": ret " + std::to_string(bad) + " error " +
           std::to_string(rec[0]) + " (flag " + std::to_string(rec[1]) + ", packet byte " + std::to_string(rec[2]) +
           ", flag seen " + std::to_string(rec[3]) + ")");
    return (int)ncclSuccess;
  });
}

}  // extern "C"
