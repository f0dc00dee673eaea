// The proxy-path harnesses of the reference's tests on this library:
//   mscclppAmdHostOffloadAllGather   test/allgather_test_host_offloading.cu:81-330 (its own proxy
//                                    handler, as the test's MyProxyService)
//   mscclppAmdPortChannelAllToAll    PortChannels built with the public host API + ProxyService
//   mscclppAmdProxyRingAllReduce     test/mscclpp-test/allreduce_test.cu:730-839 (allreduce1)
// The FIFO, proxy thread and ProxyService themselves are in channels.cpp (include/mscclpp_amd/
// {fifo,proxy,port_channel}.hpp).  Copy and token-update failures on a proxy thread are checked and
// reported (the result's correctness flag and a warning), never dropped.
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <fstream>
#include <functional>
#include <sstream>
#include <thread>

#include "comm_internal.hpp"
#include "mscclpp_amd/port_channel.hpp"

extern "C" int mscclppAmdLaunchHostOffloadKernel(int rank, int nranks, const void* fifoHandle, void* semHandles,
                                                 int handleIndex, uint64_t budget, uint32_t* err, void* stream);
extern "C" int mscclppAmdLaunchRingProxyAllReduce(int* buff, const int* scratch, int rank, int nranks, size_t nelems,
                                                  const void* channels4, void* gridBarrier, int nblocks, int nthreads,
                                                  uint64_t budget, uint32_t* err, void* stream);
extern "C" int mscclppAmdLaunchPortChannelPut(void* chans, int nchans, const uint64_t* dstOffs, const uint64_t* srcOffs,
                                              uint64_t chunk, int mode, void* stream);

namespace mscclpp_amd {
namespace host {

static double nowSec() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Drain a connection stream by busy-polling hipStreamQuery.  The reference's flush is a blocking
// stream synchronize (CudaIpcStream::sync, context.cc:37-46); the proxy thread is a dedicated
// busy-poll core anyway (proxy.cc:42-100), and a blocking wait here measured 0.1-2 ms per flush
// (interrupt wake-up) against a few microseconds of outstanding copies.
static void spinSync(hipStream_t s) {
  static const bool blocking = [] {
    const char* e = std::getenv("MSCCLPP_AMD_PROXY_BLOCKING_SYNC");
    return e && *e == '1';
  }();
  if (blocking) {
    (void)hipStreamSynchronize(s);
    return;
  }
  while (hipStreamQuery(s) == hipErrorNotReady) {
  }
}

extern "C" int mscclppAmdProxyCopy(void* dst, const void* src, size_t bytes, void* stream);

// A data trigger's copy (CudaIpcConnection::write, connection.cc:138-157): hipMemcpyAsync on the
// connection stream, as the reference does.  MSCCLPP_AMD_PROXY_COPY=kernel enqueues the CU copy
// kernel (proxy_kernels.hip) instead, a diagnostic that separates the copy engine from the
// mappings; not the default, because a copy kernel queued behind a spinning
// collective on a shared hardware queue could never run.
static hipError_t proxyCopy(void* dst, const void* src, size_t bytes, hipStream_t s) {
  static const bool kernel = [] {
    const char* e = std::getenv("MSCCLPP_AMD_PROXY_COPY");
    return e && std::string(e) == "kernel";
  }();
  if (!kernel) return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s);
  return mscclppAmdProxyCopy(dst, src, bytes, (void*)s) == 0 ? hipSuccess : hipErrorLaunchFailure;
}

// Per-peer host-driven connection: a non-blocking stream (CudaIpcStream, context.cc:16-46).
struct Conn {
  hipStream_t stream = nullptr;
};

// Stream-ordered remote token update (Host2DeviceSemaphore::signal -> CudaIpcConnection::
// updateAndSync, semaphore.cc:154-156, connection.cc:159-177).  HIP reads a pinned source when the
// copy executes, not when it is enqueued, so a single host counter could be read after a later
// increment and release a waiter before the data copies queued ahead of that later signal.  Each
// value therefore gets its own slot of a pinned ring; a slot is reused only after a stream
// synchronize has retired every copy of the previous lap.
class TokenWriter {
 public:
  TokenWriter() { HIPCHECK(hipHostMalloc((void**)&slots_, kSlots * sizeof(uint64_t), hipHostMallocDefault)); }
  ~TokenWriter() { (void)hipHostFree(slots_); }
  TokenWriter(const TokenWriter&) = delete;
  TokenWriter& operator=(const TokenWriter&) = delete;
  void signal(uint64_t* remoteToken, hipStream_t s) {
    ++value_;
    if (value_ % kSlots == 0) spinSync(s);
    uint64_t* slot = &slots_[value_ % kSlots];
    *slot = value_;
    const hipError_t e = hipMemcpyAsync(remoteToken, slot, sizeof(uint64_t), hipMemcpyHostToDevice, s);
    if (e != hipSuccess) throw HipError(e, "proxy token update (hipMemcpyAsync H2D)");
  }

 private:
  static constexpr uint64_t kSlots = 1024;
  uint64_t* slots_ = nullptr;
  uint64_t value_ = 0;
};

}  // namespace host
}  // namespace mscclpp_amd

// =============================================================================================
// Harness 1: test/allgather_test_host_offloading.cu on the C ABI (BASELINE config 1)
// =============================================================================================
extern "C" int mscclppAmdHostOffloadAllGather(ncclComm_t comm, size_t dataSize, int iters, int graphIters,
                                             double* out) {
  return guarded([&] {
    if (!comm || !out || dataSize == 0) return (int)ncclInvalidArgument;
    const int n = comm->nranks, rank = comm->rank;
    if (n < 2 || dataSize % (4 * (size_t)n)) return (int)ncclInvalidArgument;
    const size_t perRank = dataSize / n;
    const size_t nelems = dataSize / 4;
    // data: element i = i+1 in my part, 0 elsewhere (:64-79)
    // uncached (the library's pool) where the reference cudaMallocs (:66): with several ranks on one
    // GPU (tests, rehearsals) a peer's copy into cached memory can sit in another XCD's L2 when this
    // rank reads the buffer back (seen in the PortChannel harness below); across GPUs both behave alike
    int* data = (int*)allocUncached(dataSize);
    std::vector<int> h(nelems, 0);
    for (size_t i = 0; i < nelems; ++i)
      if (i / (perRank / 4) == (size_t)rank) h[i] = (int)(i + 1);
    HIPCHECK(hipMemcpy(data, h.data(), dataSize, hipMemcpyHostToDevice));
    auto peers = comm->exchange(data);
    // two Host2Device semaphore sets per peer (:86-87): inbound tokens [2][n], expected [2][n]
    uint64_t* tok = nullptr;
    uint64_t* expct = nullptr;
    HIPCHECK(hipMalloc((void**)&tok, 2 * n * 8));
    memsetSync(tok, 0, 2 * n * 8);
    HIPCHECK(hipMalloc((void**)&expct, 2 * n * 8));
    memsetSync(expct, 0, 2 * n * 8);
    auto peerTok = comm->exchange(tok);
    std::vector<std::unique_ptr<TokenWriter>> writers(2 * n);
    for (auto& w : writers) w = std::make_unique<TokenWriter>();
    std::vector<Host2DeviceSemaphoreDeviceHandle> hh(2 * n);
    for (int s = 0; s < 2; ++s)
      for (int r = 0; r < n; ++r) hh[s * n + r] = {tok + s * n + r, expct + s * n + r};
    Host2DeviceSemaphoreDeviceHandle* dh = nullptr;
    HIPCHECK(hipMalloc((void**)&dh, hh.size() * sizeof(hh[0])));
    HIPCHECK(hipMemcpy(dh, hh.data(), hh.size() * sizeof(hh[0]), hipMemcpyHostToDevice));
    // One copy stream for every peer (the reference's CUDA branch, connection.cc:126-130), not one per
    // peer (its HIP branch): HIP multiplexes a process's streams onto GPU_MAX_HW_QUEUES (4) hardware
    // queues, and a stream that lands on the queue of the spinning offload kernel never runs -- with 4
    // ranks on one GPU the per-peer form hung in the first iteration.
    hipStream_t copyStream = nullptr;
    HIPCHECK(hipStreamCreateWithFlags(&copyStream, hipStreamNonBlocking));
    std::vector<Conn> conns(n);
    for (int r = 0; r < n; ++r)
      if (r != rank) conns[r].stream = copyStream;
    uint32_t* err = nullptr;
    HIPCHECK(hipMalloc((void**)&err, 64));
    memsetSync(err, 0, 64);
    // MyProxyService::handleTrigger (:135-155)
    std::string proxyFailure;  // first copy / token failure on the proxy thread
    Proxy proxy([&](ProxyTrigger t, uint64_t) {
      if (t.fst > 0) {
        const int set = t.fst == 1 ? 0 : 1;
        try {
          for (int k = 1; k < n; ++k) {
            const int nghr = (rank + k) % n;
            const hipError_t e = hipMemcpyAsync((char*)peers[nghr] + rank * perRank, (char*)data + rank * perRank,
                                                perRank, hipMemcpyDeviceToDevice, conns[nghr].stream);
            if (e != hipSuccess) throw HipError(e, "proxy data copy (hipMemcpyAsync D2D)");
            writers[set * n + nghr]->signal((uint64_t*)peerTok[nghr] + set * n + rank, conns[nghr].stream);
          }
        } catch (const std::exception& ex) {
          if (proxyFailure.empty()) proxyFailure = ex.what();
        }
      }
      return ProxyHandlerResult::Continue;
    }, 512);
    proxy.start();
    FifoDeviceHandle fh = proxy.fifo().deviceHandle();
    hipStream_t st;
    HIPCHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const uint64_t budget = spinBudgetTicks();
    auto k = [&](int set) {
      int rc = mscclppAmdLaunchHostOffloadKernel(rank, n, &fh, dh + (set - 1) * n, set, budget, err, st);
      if (rc) throw std::runtime_error("host offload kernel launch failed");
    };
    // correctness (:258-271)
    k(1);
    HIPCHECK(hipStreamSynchronize(st));
    std::vector<int> back(nelems);
    HIPCHECK(hipMemcpy(back.data(), data, dataSize, hipMemcpyDeviceToHost));
    bool ok = true;
    for (size_t i = 0; i < nelems; ++i) ok &= back[i] == (int)(i + 1);
    comm->boot->barrier();
    // no-graph timing (:275-292)
    HIPCHECK(hipStreamSynchronize(st));
    comm->boot->barrier();
    double t0 = nowSec();
    for (int i = 0; i < iters; ++i) {
      k(1);
      k(2);
    }
    HIPCHECK(hipStreamSynchronize(st));
    comm->boot->barrier();
    double t1 = nowSec();
    out[0] = (t1 - t0) * 1e6 / iters / 2;
    // graph timing (:294-330): graphIters x (2 kernels) captured, 10 warmup replays, 10 timed
    hipGraph_t graph;
    hipGraphExec_t inst;
    HIPCHECK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
    for (int i = 0; i < graphIters; ++i) {
      k(1);
      k(2);
    }
    HIPCHECK(hipStreamEndCapture(st, &graph));
    HIPCHECK(hipGraphInstantiate(&inst, graph, nullptr, nullptr, 0));
    for (int i = 0; i < 10; ++i) HIPCHECK(hipGraphLaunch(inst, st));
    HIPCHECK(hipStreamSynchronize(st));
    comm->boot->barrier();
    t0 = nowSec();
    for (int i = 0; i < 10; ++i) HIPCHECK(hipGraphLaunch(inst, st));
    HIPCHECK(hipStreamSynchronize(st));
    t1 = nowSec();
    out[1] = (t1 - t0) * 1e6 / 10 / graphIters / 2;
    comm->boot->barrier();
    uint32_t e = 0;
    HIPCHECK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
    if (!proxyFailure.empty()) warn("host offload proxy: " + proxyFailure);
    out[2] = (ok && e == 0 && proxyFailure.empty()) ? 1.0 : 0.0;
    out[3] = (double)proxy.numaNode();
    proxy.stop();
    (void)hipStreamSynchronize(copyStream);
    (void)hipStreamDestroy(copyStream);
    (void)hipGraphExecDestroy(inst);
    (void)hipGraphDestroy(graph);
    (void)hipStreamDestroy(st);
    comm->boot->barrier();  // peers no longer touch my data / tokens
    peers = PeerBufs();     // peers free these buffers now: close our mappings of them
    peerTok = PeerBufs();
    freeDevice(err);
    freeDevice(dh);
    freeDevice(tok);
    freeDevice(expct);
    freeDevice(data);
    return (int)ncclSuccess;
  });
}

// =============================================================================================
// Harness 2: PortChannel all-to-all through the general ProxyService (port_channel.cc:117-178),
// built with the public host API the way a user kernel's channels are: Communicator::connect +
// registerMemory / sendMemory / recvMemory + ProxyService::buildAndAddSemaphore / addMemory /
// portChannel, device handles copied to the GPU.
// =============================================================================================
extern "C" int mscclppAmdPortChannelAllToAllStats(ncclComm_t comm, size_t chunk, int mode, int iters, double* out,
                                                  int outLen) {
  return guarded([&] {
    if (!comm || !out || outLen < 3 || chunk == 0 || chunk % 4 || mode < 0 || mode > 2 || iters <= 0)
      return (int)ncclInvalidArgument;
    const int n = comm->nranks, rank = comm->rank;
    if (n < 2) return (int)ncclInvalidArgument;
    const size_t bytes = chunk * n;
    // GpuBuffer, as the reference's PortChannel tests allocate (port_channel_tests.cu:209, :241):
    // uncached on AMD, so the copy engine, the peers' copies and every XCD see one copy of the data.
    // With cached hipMalloc buffers and 4 ranks sharing one GPU, a peer's copy could sit in an XCD's
    // L2 when the owner read the buffer back (1 run in 3 lost every peer's chunk on one rank).
    uint32_t* src = (uint32_t*)allocUncached(bytes);
    uint32_t* dst = (uint32_t*)allocUncached(bytes);  // zeroed
    std::vector<uint32_t> h(bytes / 4);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (uint32_t)(rank * 0x01000000u + i);  // src chunk q for peer q
    HIPCHECK(hipMemcpy(src, h.data(), bytes, hipMemcpyHostToDevice));
    double t0 = 0, t1 = 0;
    bool ok = true;
    uint32_t e = 0;
    int numa = -1;
    std::vector<double> per;  // us per iteration (HIP events)
    double maxGapUs = 0;      // longest proxy-thread gap between FIFO polls (MSCCLPP_AMD_PROXY_GAP_STATS=1)
    double stampStats[8] = {-1, -1, -1, -1, -1, -1, -1, 0};  // outLen >= 16: the trigger-stamp breakdown
    {
      Communicator cx(comm);
      ProxyService proxy;
      std::vector<std::shared_future<Connection>> cf;
      std::vector<int> peers;
      RegisteredMemory srcMem = cx.registerMemory(src, bytes, Transport::CudaIpc);
      RegisteredMemory dstMem = cx.registerMemory(dst, bytes, Transport::CudaIpc);
      std::vector<std::shared_future<RegisteredMemory>> remote;
      for (int q = 0; q < n; ++q) {
        if (q == rank) continue;
        peers.push_back(q);
        cf.push_back(cx.connect(Transport::CudaIpc, q));
        cx.sendMemory(dstMem, q);
        remote.push_back(cx.recvMemory(q));
      }
      const MemoryId srcId = proxy.addMemory(srcMem);
      std::vector<PortChannelDeviceHandle> ch;
      for (size_t i = 0; i < peers.size(); ++i) {
        const SemaphoreId sid = proxy.buildAndAddSemaphore(cx, cf[i].get());
        const MemoryId dstId = proxy.addMemory(remote[i].get());
        ch.push_back(proxy.portChannel(sid, dstId, srcId).deviceHandle());
      }
      proxy.startProxy(true);
      // channel c (peer q) moves my src chunk q to offset rank*chunk of q's dst
      std::vector<uint64_t> offs;
      for (int q : peers) offs.push_back((uint64_t)rank * chunk);
      for (int q : peers) offs.push_back((uint64_t)q * chunk);
      uint64_t* dOffs = nullptr;
      HIPCHECK(hipMalloc((void**)&dOffs, offs.size() * 8));
      HIPCHECK(hipMemcpy(dOffs, offs.data(), offs.size() * 8, hipMemcpyHostToDevice));
      PortChannelDeviceHandle* dch = nullptr;
      HIPCHECK(hipMalloc((void**)&dch, ch.size() * sizeof(ch[0])));
      HIPCHECK(hipMemcpy(dch, ch.data(), ch.size() * sizeof(ch[0]), hipMemcpyHostToDevice));
      hipStream_t st;
      HIPCHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
      // one untimed launch first: the kernel's code object loads at its first launch in a process
      // (milliseconds), and the proxy thread's first trigger of each connection opens its copy path
      if (mscclppAmdLaunchPortChannelPut(dch, (int)ch.size(), dOffs, dOffs + ch.size(), chunk, mode, st))
        throw std::runtime_error("launch");
      HIPCHECK(hipStreamSynchronize(st));
      // iters launches back to back (the ranks start together at the barrier); an event before each
      // launch and one after the last give every iteration's own duration on the stream
      std::vector<hipEvent_t> ev((size_t)iters + 1);
      for (auto& x : ev) HIPCHECK(hipEventCreate(&x));
      comm->boot->barrier();
      proxy.resetProxyPollGap();
      const int trigPerIter = (int)ch.size() * (mode == 0 ? 2 : 1);
      if (outLen >= 16) proxy.enableStamps((size_t)iters * trigPerIter);
      t0 = nowSec();
      for (int i = 0; i < iters; ++i) {
        HIPCHECK(hipEventRecord(ev[(size_t)i], st));
        if (mscclppAmdLaunchPortChannelPut(dch, (int)ch.size(), dOffs, dOffs + ch.size(), chunk, mode, st))
          throw std::runtime_error("launch");
      }
      HIPCHECK(hipEventRecord(ev[(size_t)iters], st));
      HIPCHECK(hipStreamSynchronize(st));
      t1 = nowSec();
      maxGapUs = (double)proxy.proxyMaxPollGapNs() * 1e-3;
      per.resize((size_t)iters);
      for (int i = 0; i < iters; ++i) {
        float ms = 0;
        HIPCHECK(hipEventElapsedTime(&ms, ev[(size_t)i], ev[(size_t)i + 1]));
        per[(size_t)i] = ms * 1e3;
      }
      if (outLen >= 16) {
        // where an iteration's time goes: device time from the iteration's launch
        // event to this rank's last data copy / last token update completing on the copy stream,
        // from that token update to the end of the kernel (the wait for the peers' tokens), and the
        // proxy thread's host time to submit a data copy, a token update, and a whole trigger.
        // Every rank's kernels have finished after this barrier, so every trigger of this rank has
        // been handled (a peer's last wait needed its token); the proxy thread is joined before its
        // stamps are read.
        comm->boot->barrier();
        proxy.stopProxy();
        const auto& sts = proxy.stamps();
        std::vector<double> toData, toToken, tokenToEnd, subData, subFlag, handler;
        double slowStartToToken = 0;
        const size_t slow = (size_t)(std::max_element(per.begin(), per.end()) - per.begin());
        for (int i = 0; i < iters && (size_t)(i + 1) * trigPerIter <= sts.size(); ++i) {
          float lastData = -1, lastTok = -1;
          for (int k = 0; k < trigPerIter; ++k) {
            const auto& x = sts[(size_t)i * trigPerIter + k];
            float ms = 0;
            if (x.dataEvent && hipEventElapsedTime(&ms, ev[(size_t)i], (hipEvent_t)x.dataEvent) == hipSuccess)
              lastData = std::max(lastData, ms * 1e3f);
            if (x.flagEvent && hipEventElapsedTime(&ms, ev[(size_t)i], (hipEvent_t)x.flagEvent) == hipSuccess)
              lastTok = std::max(lastTok, ms * 1e3f);
            if (x.dataNs) subData.push_back((x.dataNs - x.seenNs) * 1e-3);
            if (x.flagNs) subFlag.push_back((x.flagNs - (x.dataNs ? x.dataNs : x.seenNs)) * 1e-3);
            handler.push_back((x.doneNs - x.seenNs) * 1e-3);
          }
          if (lastData >= 0) toData.push_back(lastData);
          if (lastTok >= 0) {
            toToken.push_back(lastTok);
            tokenToEnd.push_back(per[(size_t)i] - lastTok);
            if ((size_t)i == slow) slowStartToToken = lastTok;
          }
        }
        auto med = [](std::vector<double> v) {
          if (v.empty()) return -1.0;
          std::sort(v.begin(), v.end());
          const size_t m = v.size();
          return m % 2 ? v[m / 2] : 0.5 * (v[m / 2 - 1] + v[m / 2]);
        };
        stampStats[0] = med(toData);
        stampStats[1] = med(toToken);
        stampStats[2] = med(tokenToEnd);
        stampStats[3] = med(subData);
        stampStats[4] = med(subFlag);
        stampStats[5] = med(handler);
        stampStats[6] = slowStartToToken;
        stampStats[7] = (double)sts.size();
      }
      for (auto& x : ev) (void)hipEventDestroy(x);
      comm->boot->barrier();
      // check: peer p's chunk addressed to me (its src chunk `rank`) sits at offset p*chunk of my dst
      std::vector<uint32_t> back(bytes / 4);
      HIPCHECK(hipMemcpy(back.data(), dst, bytes, hipMemcpyDeviceToHost));
      std::string bad;
      for (int p = 0; p < n; ++p) {
        if (p == rank) continue;
        size_t wrong = 0, first = 0;
        for (size_t i = 0; i < chunk / 4; ++i) {
          const size_t srcElem = (size_t)rank * (chunk / 4) + i;
          if (back[(size_t)p * (chunk / 4) + i] != (uint32_t)(p * 0x01000000u + srcElem) && wrong++ == 0) first = i;
        }
        if (wrong) {
          ok = false;
          bad += " from rank " + std::to_string(p) + ": " + std::to_string(wrong) + " words wrong (first " +
                 std::to_string(first) + ", holds " + std::to_string(back[(size_t)p * (chunk / 4) + first]) + ")";
        }
      }
      HIPCHECK(hipMemcpy(&e, comm->err, 4, hipMemcpyDeviceToHost));
      if (!ok || e)
        warn("PortChannel all-to-all mode " + std::to_string(mode) + ", rank " + std::to_string(rank) + " of " +
             std::to_string(n) + ": error word " + std::to_string(e) + bad);
      numa = proxy.proxyNumaNode();
      proxy.stopProxy();
      (void)hipStreamDestroy(st);
      freeDevice(dOffs);
      freeDevice(dch);
      comm->boot->barrier();  // every peer is done with my buffers before the mappings close
    }
    out[0] = (t1 - t0) * 1e6 / iters;
    out[1] = (ok && e == 0) ? 1.0 : 0.0;
    out[2] = (double)numa;
    if (outLen >= 7) {  // per-iteration spread: median, min, max and the slowest iteration's index
      std::vector<double> s = per;
      std::sort(s.begin(), s.end());
      const size_t m = s.size();
      out[3] = m % 2 ? s[m / 2] : 0.5 * (s[m / 2 - 1] + s[m / 2]);
      out[4] = s.front();
      out[5] = s.back();
      out[6] = (double)(std::max_element(per.begin(), per.end()) - per.begin());
    }
    if (outLen >= 8) out[7] = maxGapUs;
    if (outLen >= 16)
      for (int k = 0; k < 8; ++k) out[8 + k] = stampStats[k];
    freeDevice(src);
    freeDevice(dst);
    return (int)ncclSuccess;
  });
}

extern "C" int mscclppAmdPortChannelAllToAll(ncclComm_t comm, size_t chunk, int mode, int iters, double* out) {
  return mscclppAmdPortChannelAllToAllStats(comm, chunk, mode, iters, out, 3);
}

// =============================================================================================
// Harness 3: mscclpp-test allreduce1 -- ring RS + AG through the host proxy (allreduce_test.cu:
// 730-839; setup :1300-1400): int32, input = rank, expected n(n-1)/2 (:1172-1183).  Two PortChannels
// to the next rank (round 1: my buffer -> its scratch, round 2: my buffer -> its buffer), one
// Host2Device semaphore per (round, source).  out[0] = us per AllReduce (graph of `iters` kernels
// replayed `graphLaunches` times, common.cc:202-227), out[1] = 1 if every element is n(n-1)/2,
// out[2] = NUMA node of the proxy thread.
// =============================================================================================
extern "C" int mscclppAmdProxyRingAllReduce(ncclComm_t comm, size_t nelems, int iters, int graphLaunches, int nblocks,
                                           double* out) {
  return guarded([&] {
    if (!comm || !out || nelems == 0 || iters <= 0 || graphLaunches <= 0) return (int)ncclInvalidArgument;
    const int n = comm->nranks, rank = comm->rank;
    if (n < 2 || nelems % (size_t)n) return (int)ncclInvalidArgument;
    if (nblocks <= 0) nblocks = 24;  // runColl: 24 x 1024 (allreduce_test.cu:1122-1125)
    const size_t bytes = nelems * sizeof(int);
    const int next = (rank + 1) % n, prev = (rank + n - 1) % n;
    int* buff = (int*)allocUncached(bytes);
    int* scratch = (int*)allocUncached(bytes);
    auto peerBuff = comm->exchange(buff);
    auto peerScratch = comm->exchange(scratch);
    if (logLevel() >= 2) {
      for (void* p : {peerBuff[next], peerScratch[next]}) {
        void* b = nullptr;
        size_t sz = 0;
        const hipError_t e = hipMemGetAddressRange((hipDeviceptr_t*)&b, &sz, (hipDeviceptr_t)p);
        info("ring: peer mapping " + std::to_string((uint64_t)p) + " -> range base " + std::to_string((uint64_t)b) +
             " size " + std::to_string(sz) + " (" + hipGetErrorString(e) + ")");
      }
    }
    // tokens[round][source rank], written by the sources' proxies
    uint64_t* tok = (uint64_t*)allocUncached(2 * n * 8);
    uint64_t* expct = nullptr;
    HIPCHECK(hipMalloc((void**)&expct, 2 * n * 8));
    memsetSync(expct, 0, 2 * n * 8);
    auto peerTok = comm->exchange(tok);
    uint64_t *flushDone = nullptr, *dFlushDone = nullptr;
    TokenWriter writers[2];
    HIPCHECK(hipHostMalloc((void**)&flushDone, 2 * 64, hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(flushDone, 0, 2 * 64);
    HIPCHECK(hipHostGetDevicePointer((void**)&dFlushDone, flushDone, 0));
    uint32_t* err = nullptr;
    HIPCHECK(hipMalloc((void**)&err, 64));
    memsetSync(err, 0, 64);
    void* gb = nullptr;
    HIPCHECK(hipMalloc(&gb, 64));
    memsetSync(gb, 0, 64);
    Conn conn;
    HIPCHECK(hipStreamCreateWithFlags(&conn.stream, hipStreamNonBlocking));
    // MemoryId 0 = my buffer, 1 = next's scratch, 2 = next's buffer; semaphoreId = round
    void* mem[3] = {buff, peerScratch[next], peerBuff[next]};
    std::string proxyFailure;  // first copy / token failure on the proxy thread
    Proxy proxy([&](ProxyTrigger t, uint64_t pos) {  // ProxyService::handleTrigger
      const int round = (int)t.fields.semaphoreId;
      if (round < 0 || round > 1) return ProxyHandlerResult::Continue;
      if (t.fields.type & kTriggerData) {
        const hipError_t e = proxyCopy((char*)mem[t.fields.dstMemoryId] + t.fields.dstOffset,
                                       (char*)mem[t.fields.srcMemoryId] + t.fields.srcOffset, t.fields.size,
                                       conn.stream);
        if (e != hipSuccess && proxyFailure.empty())
          proxyFailure = "proxy copy failed: " + std::string(hipGetErrorString(e)) + " dst id " +
                         std::to_string(t.fields.dstMemoryId) + " off " + std::to_string(t.fields.dstOffset) +
                         " size " + std::to_string(t.fields.size);
      }
      if (t.fields.type & kTriggerFlag) {
        try {
          writers[round].signal((uint64_t*)peerTok[next] + round * n + rank, conn.stream);
        } catch (const std::exception& ex) {
          if (proxyFailure.empty()) proxyFailure = ex.what();
        }
      }
      if (t.fields.type & kTriggerSync) {
        spinSync(conn.stream);
        __atomic_store_n(&flushDone[round * 8], pos + 1, __ATOMIC_RELEASE);
      }
      return ProxyHandlerResult::Continue;
    }, 512);
    proxy.start();
    const uint64_t budget = spinBudgetTicks();
    PortChannelDeviceHandle ch[4] = {};
    for (int round = 0; round < 2; ++round) {
      PortChannelDeviceHandle& snd = ch[round * 2];      // to next
      PortChannelDeviceHandle& rcv = ch[round * 2 + 1];  // from prev: only its semaphore is used
      snd.semaphoreId_ = (uint32_t)round;
      snd.src_ = 0;
      snd.dst_ = (uint32_t)(1 + round);
      snd.fifo_ = proxy.fifo().deviceHandle(budget, err);
      snd.flushDonePos_ = dFlushDone + round * 8;
      snd.semaphore_ = {tok + round * n + next, expct + round * n + next, budget, err};
      rcv = snd;
      rcv.semaphore_ = {tok + round * n + prev, expct + round * n + prev, budget, err};
    }
    hipStream_t st;
    HIPCHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    std::vector<int> init(nelems, rank);
    auto reset = [&] { HIPCHECK(hipMemcpy(buff, init.data(), bytes, hipMemcpyHostToDevice)); };
    auto launch = [&] {
      int rc = mscclppAmdLaunchRingProxyAllReduce(buff, scratch, rank, n, nelems, ch, gb, nblocks, 1024, budget, err, st);
      if (rc) throw std::runtime_error("ring kernel launch failed: " + std::to_string(rc));
    };
    // correctness first (checkData, common.cc:346-360)
    reset();
    comm->boot->barrier();
    launch();
    HIPCHECK(hipStreamSynchronize(st));
    std::vector<int> back(nelems);
    HIPCHECK(hipMemcpy(back.data(), buff, bytes, hipMemcpyDeviceToHost));
    bool ok = true;
    const int expected = n * (n - 1) / 2;
    size_t nbad = 0, firstBad = nelems;
    for (size_t i = 0; i < nelems; ++i)
      if (back[i] != expected && nbad++ == 0) firstBad = i;
    ok = nbad == 0;
    if (!ok) {
      uint32_t e0 = 0;
      (void)hipMemcpy(&e0, err, 4, hipMemcpyDeviceToHost);
      // where did the peer's contribution go?  my scratch at the first bad element, my tokens
      int sc = -1;
      (void)hipMemcpy(&sc, scratch + firstBad, 4, hipMemcpyDeviceToHost);
      std::vector<uint64_t> tk(2 * (size_t)n);
      (void)hipMemcpy(tk.data(), tok, tk.size() * 8, hipMemcpyDeviceToHost);
      std::string ts;
      for (auto t : tk) ts += std::to_string(t) + " ";
      warn("proxy ring allreduce rank " + std::to_string(rank) + ": scratch at first bad = " + std::to_string(sc) +
           ", tokens [round][src] = " + ts + ", buff " + std::to_string((uint64_t)buff) + " scratch " +
           std::to_string((uint64_t)scratch) + " peerScratch[next] " + std::to_string((uint64_t)peerScratch[next]) +
           " peerBuff[next] " + std::to_string((uint64_t)peerBuff[next]));
      warn("proxy ring allreduce rank " + std::to_string(rank) + ": " + std::to_string(nbad) + " wrong of " +
           std::to_string(nelems) + ", first at " + std::to_string(firstBad) + " = " +
           std::to_string(back[firstBad]) + ", device error " + std::to_string(e0));
    }
    comm->boot->barrier();
    // benchTime: iters launches in one graph, graphLaunches replays after a barrier
    hipGraph_t graph;
    hipGraphExec_t inst;
    HIPCHECK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
    for (int i = 0; i < iters; ++i) launch();
    HIPCHECK(hipStreamEndCapture(st, &graph));
    HIPCHECK(hipGraphInstantiate(&inst, graph, nullptr, nullptr, 0));
    comm->boot->barrier();
    const double t0 = nowSec();
    for (int l = 0; l < graphLaunches; ++l) HIPCHECK(hipGraphLaunch(inst, st));
    HIPCHECK(hipStreamSynchronize(st));
    const double t1 = nowSec();
    comm->boot->barrier();
    uint32_t e = 0;
    HIPCHECK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
    out[0] = (t1 - t0) * 1e6 / iters / graphLaunches;
    if (!proxyFailure.empty()) warn("ring proxy: " + proxyFailure);
    out[1] = (ok && e == 0 && proxyFailure.empty()) ? 1.0 : 0.0;
    out[2] = (double)proxy.numaNode();
    proxy.stop();
    (void)hipStreamSynchronize(conn.stream);
    (void)hipStreamDestroy(conn.stream);
    (void)hipGraphExecDestroy(inst);
    (void)hipGraphDestroy(graph);
    (void)hipStreamDestroy(st);
    comm->boot->barrier();  // peers no longer touch my buffers / tokens
    peerBuff = peerScratch = peerTok = PeerBufs();
    freeDevice(gb);
    freeDevice(err);
    (void)hipHostFree(flushDone);
    freeDevice(tok);
    freeDevice(expct);
    freeDevice(scratch);
    freeDevice(buff);
    return (int)ncclSuccess;
  });
}
