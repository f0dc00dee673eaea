// Self-tests of the MemoryChannel device surface on one GPU: two in-process "ranks" (blocks 0 and 1
// of one launch), each with its own buffer, packet buffer and semaphore tokens, connected by
// MemoryChannelDeviceHandles whose dst_ points at the other rank's memory.
//
//  mode 0: LL16 packet ping-pong  (test/mp_unit/memory_channel_tests.cu:286-338)
//  mode 1: LL8 packet ping-pong   (memory_channel_tests.cu:246-284)
//  mode 2: put + signal / wait + get round trip (memory_channel_tests.cu put/get/signal tests)
#include "common.hpp"
#include "mscclpp_amd/memory_channel_device.hpp"

namespace mscclpp_amd {

__global__ void memChanSelfTestKernel(MemoryChannelDeviceHandle* chans, int* b0, int* b1, int nElem, int nTries,
                                      int mode, int* ret) {
  const int rank = blockIdx.x;
  MemoryChannelDeviceHandle& ch = chans[rank];
  int* sendBuff = rank == 0 ? b0 : b1;
  const int putOffset = rank == 0 ? 0 : 10000000;
  const int getOffset = rank == 0 ? 10000000 : 0;
  if (mode == 3 || mode == 4) {
    // a packet that never comes: rank 0 unpacks LL16 (mode 3) / LL8 (mode 4) packets of flag 7 that
    // rank 1 never puts; the wait ends at the handle's budget with the error record filled in
    if (rank == 0) {
      if (mode == 3)
        ch.unpackPackets<LL16Packet>(0, 0, nElem * sizeof(int), threadIdx.x, blockDim.x, 7u);
      else
        ch.unpackPackets<LL8Packet>(0, 0, nElem * sizeof(int), threadIdx.x, blockDim.x, 7u);
    }
    return;
  }
  if (mode <= 1) {
    for (int i = 0; i < nTries; ++i) {
      const uint32_t flag = (uint32_t)i + 1;
      if ((rank ^ (i & 1)) == 0) {
        for (int j = threadIdx.x; j < nElem; j += blockDim.x) sendBuff[j] = putOffset + i + j;
        __syncthreads();
        if (mode == 0)
          ch.putPackets<LL16Packet>(0, 0, nElem * sizeof(int), threadIdx.x, blockDim.x, flag);
        else
          ch.putPackets<LL8Packet>(0, 0, nElem * sizeof(int), threadIdx.x, blockDim.x, flag);
      } else {
        if (mode == 0)
          ch.unpackPackets<LL16Packet>(0, 0, nElem * sizeof(int), threadIdx.x, blockDim.x, flag);
        else
          ch.unpackPackets<LL8Packet>(0, 0, nElem * sizeof(int), threadIdx.x, blockDim.x, flag);
        __syncthreads();
        for (int j = threadIdx.x; j < nElem; j += blockDim.x)
          if (sendBuff[j] != getOffset + i + j) atomicAdd(ret, 1);
      }
      __syncthreads();
    }
    return;
  }
  // mode 2: each rank writes its half into the peer's buffer, signals, waits for the peer's
  // signal, checks the half it received, then gets the peer's own half back and checks it.
  const int half = nElem / 2;
  for (int i = 0; i < nTries; ++i) {
    for (int j = threadIdx.x; j < half; j += blockDim.x) sendBuff[rank * half + j] = putOffset + i + j;
    __syncthreads();
    ch.put((uint64_t)rank * half * 4, (uint64_t)half * 4, threadIdx.x, blockDim.x);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      ch.signal();
      ch.wait();
    }
    __syncthreads();
    const int peer = 1 - rank;
    for (int j = threadIdx.x; j < half; j += blockDim.x)
      if (sendBuff[peer * half + j] != getOffset + i + j) atomicAdd(ret, 1);
    __syncthreads();
    if (threadIdx.x == 0) {  // both ranks are done reading before the next round overwrites
      ch.signal();
      ch.wait();
    }
    __syncthreads();
  }
}

// ---- two-process packet ping-pong (the reference's latency measurement) ------------------------
// test/mp_unit/memory_channel_tests.cu:98-107 with kernelMemLL8/LL16PacketPingPong (:246-325): rank 0
// and rank 1 take turns, round i's sender (rank == i & 1) fills its buffer and putPackets it into the
// peer's packet buffer with flag flagBase + i + 1, the receiver unpackPackets and checks.  One
// 1024-lane workgroup per rank.
__global__ void memChanPingPongKernel(MemoryChannelDeviceHandle ch, int* buff, int rank, int nElem, int nTries,
                                      uint32_t flagBase, int ll8, int* ret) {
  // Lane t fills, and after the receive checks, exactly the words its own packets carry (LL8
  // packet t: word t; LL16 packet t: words 2t, 2t + 1), so no workgroup barrier is needed between
  // the fill and the put or between the unpack and the check -- the reference kernels' pattern.
  volatile int* sendBuff = buff;
  const int putOffset = rank == 0 ? 0 : 10000000;
  const int getOffset = rank == 0 ? 10000000 : 0;
  const int wordsPerPacket = ll8 ? 1 : 2;
  const int nPkt = nElem / wordsPerPacket;
  for (int i = 0; i < nTries; ++i) {
    const uint32_t flag = flagBase + (uint32_t)i + 1;
    if ((rank ^ (i & 1)) == 0) {
      for (int t = threadIdx.x; t < nPkt; t += blockDim.x)
        for (int w = 0; w < wordsPerPacket; ++w) {
          const int j = t * wordsPerPacket + w;
          sendBuff[j] = putOffset + i + j;
        }
      if (ll8)
        ch.putPackets<LL8Packet>(0, 0, (uint64_t)nElem * 4, threadIdx.x, blockDim.x, flag);
      else
        ch.putPackets<LL16Packet>(0, 0, (uint64_t)nElem * 4, threadIdx.x, blockDim.x, flag);
    } else {
      if (ll8)
        ch.unpackPackets<LL8Packet>(0, 0, (uint64_t)nElem * 4, threadIdx.x, blockDim.x, flag);
      else
        ch.unpackPackets<LL16Packet>(0, 0, (uint64_t)nElem * 4, threadIdx.x, blockDim.x, flag);
      for (int t = threadIdx.x; t < nPkt; t += blockDim.x)
        for (int w = 0; w < wordsPerPacket; ++w) {
          const int j = t * wordsPerPacket + w;
          if (sendBuff[j] != getOffset + i + j) *ret = 1;
        }
    }
    __syncthreads();
  }
}

// ---- buffers beyond 4 GiB (the primitives' buffer resources are rebased window by window) -------
// word i of the pattern: distinct for words 2^30 apart, so a copy that wrapped at 4 GiB shows
__device__ __forceinline__ uint32_t bigPattern(uint64_t i) {
  return (uint32_t)(i * 2654435761ull) ^ (uint32_t)(i >> 30) * 0x9E3779B9u ^ 0x5bd1e995u;
}
__global__ void bigFillKernel(uint32_t* p, uint64_t words) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < words; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = bigPattern(i);
}
__global__ void bigCountKernel(const uint32_t* p, uint64_t words, unsigned long long* bad) {
  unsigned long long n = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < words; i += (uint64_t)gridDim.x * blockDim.x)
    n += p[i] != bigPattern(i);
  if (n) atomicAdd(bad, n);
}
// op 0 put, 1 get, 2 putPackets<LL16>, 3 unpackPackets<LL16>, 4 putPackets<LL8>, 5 unpackPackets<LL8>;
// the whole grid is one "thread group" of the primitive (threadId = flat id, numThreads = grid size)
__global__ void bigChannelKernel(MemoryChannelDeviceHandle ch, uint64_t bytes, int op) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x, nt = gridDim.x * blockDim.x;
  switch (op) {
    case 0: ch.put(0, bytes, tid, nt); break;
    case 1: ch.get(0, bytes, tid, nt); break;
    case 2: ch.putPackets<LL16Packet>(0, 0, bytes, tid, nt, 1u); break;
    case 3: ch.unpackPackets<LL16Packet>(0, 0, bytes, tid, nt, 1u); break;
    case 4: ch.putPackets<LL8Packet>(0, 0, bytes, tid, nt, 2u); break;
    default: ch.unpackPackets<LL8Packet>(0, 0, bytes, tid, nt, 2u); break;
  }
}

}  // namespace mscclpp_amd

using namespace mscclpp_amd;

// put / get / putPackets + unpackPackets (LL16, LL8) of `bytes` (a multiple of 16; > 4 GiB is the
// point) on one GPU: a patterned source, a "peer" buffer and a packet buffer.  bad[0..3]: words that
// differ from the pattern after put (peer), get (back into a cleared local), LL16 and LL8 round trips.
extern "C" int mscclppAmdMemChannelBigTest(uint64_t bytes, int nblocks, unsigned long long* bad, uint32_t* devErr) {
  if (!bad || !devErr || bytes == 0 || bytes % 16 || nblocks <= 0 || nblocks > 4096) return 4;
  const uint64_t words = bytes / 4;
  uint32_t *src = nullptr, *peer = nullptr, *local = nullptr, *err = nullptr;
  void* pk = nullptr;
  unsigned long long* dbad = nullptr;
  int rc = 0;
  const dim3 grid(nblocks), block(256);
  auto count = [&](const uint32_t* p, int k) {
    if (hipMemset(dbad + k, 0, 8) != hipSuccess) return false;
    hipLaunchKernelGGL(bigCountKernel, dim3(1024), block, 0, 0, p, words, dbad + k);
    return hipGetLastError() == hipSuccess;
  };
  auto run = [&](void* dst, void* srcp, void* pkt, int op) {
    MemoryChannelDeviceHandle h{};
    h.semaphore_ = {nullptr, nullptr, nullptr, 200000000ull /* 2 s */, err};
    h.dst_ = dst;
    h.src_ = srcp;
    h.packetBuffer_ = pkt;
    hipLaunchKernelGGL(bigChannelKernel, grid, block, 0, 0, h, bytes, op);
    return hipGetLastError() == hipSuccess;
  };
#define CK(x)              \
  if (!(x)) {              \
    rc = 1;                \
    goto done;             \
  }
  CK(hipMalloc((void**)&src, bytes) == hipSuccess);
  CK(hipMalloc((void**)&peer, bytes) == hipSuccess);
  CK(hipMalloc((void**)&local, bytes) == hipSuccess);
  CK(hipMalloc(&pk, 2 * bytes) == hipSuccess);
  CK(hipMalloc((void**)&dbad, 4 * 8) == hipSuccess);
  CK(hipMalloc((void**)&err, 16) == hipSuccess);
  CK(hipMemset(err, 0, 16) == hipSuccess);
  CK(hipMemset(peer, 0, bytes) == hipSuccess);
  hipLaunchKernelGGL(bigFillKernel, dim3(1024), block, 0, 0, src, words);
  CK(hipGetLastError() == hipSuccess);
  CK(run(peer, src, nullptr, 0));  // put: src -> peer
  CK(count(peer, 0));
  CK(hipMemset(local, 0, bytes) == hipSuccess);
  CK(run(peer, local, nullptr, 1));  // get: peer -> local
  CK(count(local, 1));
  CK(hipMemset(pk, 0, 2 * bytes) == hipSuccess);
  CK(hipMemset(local, 0, bytes) == hipSuccess);
  CK(run(pk, src, nullptr, 2));   // putPackets<LL16>: src -> packets
  CK(run(nullptr, local, pk, 3));  // unpackPackets<LL16>: packets -> local
  CK(count(local, 2));
  CK(hipMemset(local, 0, bytes) == hipSuccess);
  CK(run(pk, src, nullptr, 4));
  CK(run(nullptr, local, pk, 5));
  CK(count(local, 3));
  CK(hipDeviceSynchronize() == hipSuccess);
  CK(hipMemcpy(bad, dbad, 4 * 8, hipMemcpyDeviceToHost) == hipSuccess);
  CK(hipMemcpy(devErr, err, 4, hipMemcpyDeviceToHost) == hipSuccess);
done:
#undef CK
  (void)hipDeviceSynchronize();
  for (void* p : {(void*)src, (void*)peer, (void*)local, pk, (void*)dbad, (void*)err})
    if (p) (void)hipFree(p);
  return rc;
}

// One rank's side of the ping-pong; `handle` points at a host MemoryChannelDeviceHandle (dst_ = the
// peer's packet buffer, src_ = buff, packetBuffer_ = this rank's packet buffer).
extern "C" int mscclppAmdLaunchMemChannelPingPong(const void* handle, int* buff, int rank, int nElem, int nTries,
                                                  uint32_t flagBase, int ll8, int* ret, void* stream) {
  if (!handle || !buff || !ret || rank < 0 || rank > 1 || nElem <= 0 || nElem % 2 || nTries <= 0) return 4;
  const MemoryChannelDeviceHandle h = *static_cast<const MemoryChannelDeviceHandle*>(handle);
  hipLaunchKernelGGL(memChanPingPongKernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, h, buff, rank, nElem, nTries,
                     flagBase, ll8, ret);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// Returns 0 on success, the mismatch count in *failures, any device error code in *devErr.  Modes 3
// and 4 (a packet that never arrives, LL16 / LL8) copy the whole error record into devErr[0..3].
extern "C" int mscclppAmdMemChannelSelfTest(int mode, int nElem, int nTries, int* failures, uint32_t* devErr) {
  if (!failures || !devErr || nElem <= 0 || nElem % 2 || mode < 0 || mode > 4) return 4;
  const size_t bytes = (size_t)nElem * 4;
  int *b[2] = {nullptr, nullptr}, *ret = nullptr;
  void* pk[2] = {nullptr, nullptr};
  uint64_t *tok = nullptr, *exp = nullptr;
  uint32_t* err = nullptr;
  MemoryChannelDeviceHandle* dch = nullptr;
  int rc = 0;
#define CK(x)                   \
  if ((x) != hipSuccess) {      \
    rc = 1;                     \
    goto done;                  \
  }
  for (int r = 0; r < 2; ++r) {
    CK(hipMalloc((void**)&b[r], bytes));
    CK(hipMemset(b[r], 0, bytes));
    CK(hipExtMallocWithFlags(&pk[r], bytes * 4, hipDeviceMallocUncached));
    CK(hipMemset(pk[r], 0, bytes * 4));
  }
  CK(hipExtMallocWithFlags((void**)&tok, 64, hipDeviceMallocUncached));
  CK(hipMemset(tok, 0, 64));
  CK(hipMalloc((void**)&exp, 64));
  CK(hipMemset(exp, 0, 64));
  CK(hipMalloc((void**)&ret, 4));
  CK(hipMemset(ret, 0, 4));
  CK(hipMalloc((void**)&err, 16));  // code + the three detail words of a packet timeout
  CK(hipMemset(err, 0, 16));
  {
    MemoryChannelDeviceHandle h[2];
    for (int r = 0; r < 2; ++r) {
      const int p = 1 - r;
      h[r].semaphore_ = {tok + r, tok + p, exp + r, mode >= 3 ? 2000000ull /* 20 ms */ : 200000000ull /* 2 s */, err};
      // packet modes: dst_ = peer's packet buffer; mode 2: dst_ = peer's data buffer
      h[r].dst_ = mode != 2 ? pk[p] : (void*)b[p];
      h[r].src_ = b[r];
      h[r].packetBuffer_ = pk[r];
    }
    CK(hipMalloc((void**)&dch, sizeof(h)));
    CK(hipMemcpy(dch, h, sizeof(h), hipMemcpyHostToDevice));
  }
  hipLaunchKernelGGL(memChanSelfTestKernel, dim3(2), dim3(256), 0, 0, dch, b[0], b[1], nElem, nTries, mode, ret);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(failures, ret, 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(devErr, err, mode >= 3 ? 16 : 4, hipMemcpyDeviceToHost));
done:
#undef CK
  for (int r = 0; r < 2; ++r) {
    if (b[r]) (void)hipFree(b[r]);
    if (pk[r]) (void)hipFree(pk[r]);
  }
  if (tok) (void)hipFree(tok);
  if (exp) (void)hipFree(exp);
  if (ret) (void)hipFree(ret);
  if (err) (void)hipFree(err);
  if (dch) (void)hipFree(dch);
  return rc;
}
