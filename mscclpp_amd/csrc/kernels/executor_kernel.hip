// Device interpreter for execution plans (the reference's DSL executor).
//
// Reference: src/core/include/execution_kernel.hpp:64-842 (executionKernel and the handle*
// functions).  One workgroup runs one plan threadblock: it copies its threadblock plan into LDS,
// then executes the operations in order.  Operation semantics, offsets and sum orders follow the
// reference handler by handler (each cites its source lines); the machinery is gfx950's own:
//  * remote stores are system-scope write-through (sc0 sc1) and remote loads system-scope, so peer
//    GPUs see and supply current bytes over xGMI without relying on L2 state;
//  * packets are written with one 16-byte (LL16) or 8-byte (LL8) store and polled with bounded,
//    time-limited spins that report to the executor's error word;
//  * `nop` drains this wave's stores before the workgroup barrier (a workgroup barrier alone does
//    not order another wave's in-flight stores on CDNA), so the signal that follows publishes them;
//  * NVLS / multimem operations do not exist on MI355X and are rejected when the plan is loaded.
#include "common.hpp"
#include "executor_common.hpp"

namespace mscclpp_amd {
namespace exec {

struct Ctx {
  uint8_t* input;
  uint8_t* output;
  uint8_t* scratch;       // raw scratch base
  uint64_t scratchOffset; // active half (double scratch) in bytes
  uint64_t scratchChunk;  // reuse-scratch chunk size
  uint32_t flag;
  uint64_t budget;
  uint32_t* err;
  Syncer* syncers;
  Sem* sems;
  const TbHeader* h;
};

__device__ __forceinline__ uint8_t* getBuffer(const Ctx& c, uint8_t type) {
  if (type == kInput) return c.input;
  if (type == kOutput) return c.output;
  if (type == kScratch) return c.scratch + c.scratchOffset;
  return nullptr;
}

template <bool ReuseScratch>
__device__ __forceinline__ uint64_t getOffset(const Ctx& c, uint8_t type, uint64_t offset) {
  if constexpr (!ReuseScratch) return offset;
  else return type == kScratch ? offset % c.scratchChunk : offset;
}

__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }

// ---- byte movement ---------------------------------------------------------------------------

// copy (copy_device.hpp:34-128): 16-byte vectors when both ends allow, then 4-byte words, then
// bytes.  `RemoteDst` / `RemoteSrc` select system-scope accesses for the side behind a channel.
template <bool RemoteDst, bool RemoteSrc>
__device__ void copyBytes(uint8_t* dst, const uint8_t* src, uint64_t bytes, uint32_t tid, uint32_t nthreads) {
  uint64_t done = 0;
  if ((((uintptr_t)dst | (uintptr_t)src) & 15) == 0) {
    const uint64_t n16 = bytes / 16;
    for_each_strided<16>(n16, tid, nthreads, [&](uint64_t, uint64_t w0, uint32_t off) {
      const auto rs = make_rsrc(src + w0 * 16);
      const auto rd = make_rsrc(dst + w0 * 16);
      u32x4 v = RemoteSrc ? load16<kSystem>(rs, off) : load16<kPlain>(rs, off);
      if (RemoteDst) store16<kSystem>(rd, off, v);
      else store16<kPlain>(rd, off, v);
    });
    done = n16 * 16;
  }
  if ((((uintptr_t)(dst + done) | (uintptr_t)(src + done)) & 3) == 0) {
    const uint64_t n4 = (bytes - done) / 4;
    const uint32_t* s4 = (const uint32_t*)(src + done);
    uint32_t* d4 = (uint32_t*)(dst + done);
    for (uint64_t i = tid; i < n4; i += nthreads) {
      uint32_t v = RemoteSrc ? __hip_atomic_load(const_cast<uint32_t*>(s4 + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                             : s4[i];
      if (RemoteDst) __hip_atomic_store(d4 + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      else d4[i] = v;
    }
    done += n4 * 4;
  }
  for (uint64_t i = done + tid; i < bytes; i += nthreads) dst[i] = src[i];
}

// ---- reductions over 32-bit words --------------------------------------------------------------

template <int DT>
__device__ __forceinline__ uint32_t red(uint8_t op, uint32_t a, uint32_t b) {
  return op == kMin ? reduce_word<DT, kMin>(a, b) : reduce_word<DT, kSum>(a, b);
}
template <int DT>
__device__ __forceinline__ u32x4 red4(uint8_t op, u32x4 a, u32x4 b) {
  return op == kMin ? reduce4<DT, kMin>(a, b) : reduce4<DT, kSum>(a, b);
}

__device__ __forceinline__ u32x4 ld16(const uint8_t* p, bool remote) {
  const auto r = make_rsrc(p);
  return remote ? load16<kSystem>(r, 0) : load16<kPlain>(r, 0);
}
__device__ __forceinline__ void st16(uint8_t* p, u32x4 v, bool remote) {
  const auto r = make_rsrc(p);
  if (remote) store16<kSystem>(r, 0, v);
  else store16<kPlain>(r, 0, v);
}
__device__ __forceinline__ uint32_t ld4(const uint8_t* p, bool remote) {
  return remote ? __hip_atomic_load(const_cast<uint32_t*>((const uint32_t*)p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                : *(const uint32_t*)p;
}
__device__ __forceinline__ void st4(uint8_t* p, uint32_t v, bool remote) {
  if (remote) __hip_atomic_store((uint32_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  else *(uint32_t*)p = v;
}

// ---- packets ----------------------------------------------------------------------------------

template <bool LL16>
struct Pkt {
  static constexpr uint32_t kPayload = LL16 ? 8 : 4;  // PacketPayload<PacketType>
  static constexpr uint32_t kBytes = LL16 ? 16 : 8;   // sizeof(PacketType)
  // write packet `i` of the packet array at `base` (system scope: the array may be a peer's)
  __device__ static __forceinline__ void write(uint8_t* base, uint64_t i, uint32_t w0, uint32_t w1, uint32_t flag) {
    if constexpr (LL16) reinterpret_cast<LL16Packet*>(base)[i].write(w0, w1, flag);
    else reinterpret_cast<LL8Packet*>(base)[i].write(w0, flag);
  }
  __device__ static __forceinline__ void read(const uint8_t* base, uint64_t i, uint32_t flag, uint32_t& w0, uint32_t& w1,
                                              const Ctx& c) {
    if constexpr (LL16) {
      reinterpret_cast<const LL16Packet*>(base)[i].read(flag, w0, w1, c.budget, c.err);
    } else {
      reinterpret_cast<const LL8Packet*>(base)[i].read(flag, w0, c.budget, c.err);
      w1 = 0;
    }
  }
  __device__ static __forceinline__ void loadPayload(const uint8_t* p, uint64_t i, uint32_t& w0, uint32_t& w1) {
    const uint32_t* q = (const uint32_t*)(p + i * kPayload);
    w0 = q[0];
    w1 = LL16 ? q[1] : 0;
  }
  __device__ static __forceinline__ void storePayload(uint8_t* p, uint64_t i, uint32_t w0, uint32_t w1) {
    uint32_t* q = (uint32_t*)(p + i * kPayload);
    q[0] = w0;
    if constexpr (LL16) q[1] = w1;
  }
};

// copyToPackets (copy_device.hpp:156-184): payload element i -> packet i
template <bool LL16>
__device__ void copyToPackets(uint8_t* dst, const uint8_t* src, uint64_t bytes, uint32_t flag) {
  using P = Pkt<LL16>;
  const uint64_t n = bytes / P::kPayload;
  for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) {
    uint32_t w0, w1;
    P::loadPayload(src, i, w0, w1);
    P::write(dst, i, w0, w1, flag);
  }
}

// ---- handlers (execution_kernel.hpp) ----------------------------------------------------------

__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// handleNop (:85)
__device__ __forceinline__ void handleNop() {
  drain();
  __syncthreads();
}

// handleBarrier (:87-90) over DeviceSyncer (concurrency_device.hpp:44-61): a monotonic arrival
// counter; the n workgroups of one barrier instance leave once the count reaches the next multiple
// of n.
__device__ void handleBarrier(const Op& op, const Ctx& c) {
  drain();
  __syncthreads();
  const uint32_t n = op.nThreadBlocks;
  if (n > 1 && threadIdx.x == 0) {
    uint64_t* cnt = &c.syncers[op.syncer].count;
    const uint64_t old = add_release_agent(cnt, 1);
    const uint64_t target = (old / n + 1) * n;
    SpinGuard g(c.budget);
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (g.expired()) {
        report_error_detail(c.err, kErrSemaphoreTimeout, 0xB0000000u | op.syncer, blockIdx.x, (uint32_t)target);
        break;
      }
    }
    acquire_agent();
  }
  __syncthreads();
}

// handleSignal / handleWait (:92-128): lanes tid < nChannels act on channel chan[tid].  In the
// reference the other lanes run on and plans add a nop where the workgroup must wait; here a
// signal first drains every wave's stores and meets at a workgroup barrier, and a wait ends with
// one, so a signal publishes the whole workgroup's writes and nothing reads ahead of a wait even
// in a plan without those nops (the results are the same; only stragglers are held).
template <bool Relaxed>
__device__ __forceinline__ void handleSignal(const Op& op, const Ctx& c) {
  const uint32_t tid = threadIdx.x;
  if (!Relaxed) {
    drain();
    __syncthreads();
  }
  if (tid < op.nChannels) {
    const Chan& ch = c.h->ch[op.chan[tid]];
    if (Relaxed) add_relaxed_sys(ch.remoteToken, 1);
    else add_release_sys(ch.remoteToken, 1);
  }
}

template <bool Relaxed>
__device__ __forceinline__ void handleWait(const Op& op, const Ctx& c) {
  const uint32_t tid = threadIdx.x;
  if (tid < op.nChannels) {
    const Chan& ch = c.h->ch[op.chan[tid]];
    const uint64_t want = __hip_atomic_fetch_add(ch.expected, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
    SpinGuard g(c.budget);
    while (ld_relaxed_sys(ch.inbound) < want) {
      if (g.expired()) {
        report_error_detail(c.err, kErrSemaphoreTimeout, op.chan[tid], blockIdx.x, (uint32_t)want);
        break;
      }
    }
    if (!Relaxed) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      drain();
    }
  }
  if (!Relaxed) __syncthreads();
}

// handlePut (:144-185), memory channels (put / pws / pwsf move the same bytes; the signal of
// pws / pwsf exists only on port channels there)
template <bool ReuseScratch>
__device__ void handlePut(const Op& op, const Ctx& c, uint64_t offset, uint64_t unitSize) {
  uint8_t* src = getBuffer(c, op.inRef[0]);
  for (uint32_t i = 0; i < op.nOutputs; ++i) {
    const uint8_t r = op.outRef[i];
    const uint64_t dstOff = op.outOff[i] + getOffset<ReuseScratch>(c, c.h->remoteType[r], offset);
    const uint64_t srcOff = op.inOff[i] + getOffset<ReuseScratch>(c, op.inRef[i], offset);
    if (op.outSize[i] <= offset) continue;
    const uint64_t size = umin64(op.outSize[i] - offset, unitSize);
    copyBytes<true, false>((uint8_t*)c.h->remotePtr[r] + dstOff, src + srcOff, size, threadIdx.x, blockDim.x);
  }
}

// handleGet (:129-142).  Kept exactly as the reference addresses it: the local side is indexed by
// the source offset and the remote side by the destination offset.
template <bool ReuseScratch>
__device__ void handleGet(const Op& op, const Ctx& c, uint64_t offset, uint64_t unitSize) {
  for (uint32_t i = 0; i < op.nInputs; ++i) {
    const uint8_t r = op.inRef[i];
    const uint64_t dstOff = op.outOff[i] + getOffset<ReuseScratch>(c, op.outRef[i], offset);
    const uint64_t srcOff = op.inOff[i] + getOffset<ReuseScratch>(c, c.h->remoteType[r], offset);
    if (op.inSize[i] <= offset) continue;
    const uint64_t size = umin64(op.inSize[i] - offset, unitSize);
    copyBytes<false, true>(getBuffer(c, op.outRef[i]) + srcOff, (const uint8_t*)c.h->remotePtr[r] + dstOff, size,
                           threadIdx.x, blockDim.x);
  }
}

// handleCopy (:509-520)
template <bool ReuseScratch>
__device__ void handleCopy(const Op& op, const Ctx& c, uint64_t offset, uint64_t unitSize) {
  if (op.inSize[0] <= offset) return;
  const uint64_t size = umin64(op.inSize[0] - offset, unitSize);
  const uint64_t dstOff = op.outOff[0] + getOffset<ReuseScratch>(c, op.outRef[0], offset);
  const uint64_t srcOff = op.inOff[0] + getOffset<ReuseScratch>(c, op.inRef[0], offset);
  copyBytes<false, false>(getBuffer(c, op.outRef[0]) + dstOff, getBuffer(c, op.inRef[0]) + srcOff, size, threadIdx.x,
                          blockDim.x);
}

// handleReadReduceSend (:187-260): out = in (+) remote inputs in listed order; optionally written
// to the remote outputs too.
template <int DT, bool ReuseScratch, bool SendToRemote>
__device__ void handleReadReduceSend(const Op& op, const Ctx& c, uint64_t offset, uint64_t unitSize) {
  if (op.inSize[0] <= offset) return;
  const uint64_t size = umin64(op.inSize[0] - offset, unitSize);
  const uint8_t* in = getBuffer(c, op.inRef[0]) + op.inOff[0] + getOffset<ReuseScratch>(c, op.inRef[0], offset);
  uint8_t* out = getBuffer(c, op.outRef[0]) + op.outOff[0] + getOffset<ReuseScratch>(c, op.outRef[0], offset);
  const uint32_t nRemoteIn = op.nInputs - 1, nRemoteOut = op.nOutputs - 1;
  const uint8_t* rin[kMaxBuffersPerOp];
  uint8_t* rout[kMaxBuffersPerOp];
  for (uint32_t k = 0; k < nRemoteIn; ++k) {
    const uint8_t r = op.inRef[k + 1];
    rin[k] = (const uint8_t*)c.h->remotePtr[r] + op.inOff[k + 1] + getOffset<ReuseScratch>(c, c.h->remoteType[r], offset);
  }
  for (uint32_t k = 0; k < nRemoteOut; ++k) {
    const uint8_t r = op.outRef[k + 1];
    rout[k] = (uint8_t*)c.h->remotePtr[r] + op.outOff[k + 1] + getOffset<ReuseScratch>(c, c.h->remoteType[r], offset);
  }
  const uint64_t n16 = size / 16;
  for (uint64_t i = threadIdx.x; i < n16; i += blockDim.x) {
    u32x4 acc = ld16(in + i * 16, false);
    for (uint32_t k = 0; k < nRemoteIn; ++k) acc = red4<DT>(op.reduceOp, acc, ld16(rin[k] + i * 16, true));
    st16(out + i * 16, acc, false);
    if constexpr (SendToRemote)
      for (uint32_t k = 0; k < nRemoteOut; ++k) st16(rout[k] + i * 16, acc, true);
  }
  for (uint64_t b = n16 * 16 + threadIdx.x * 4; b + 4 <= size; b += (uint64_t)blockDim.x * 4) {
    uint32_t acc = ld4(in + b, false);
    for (uint32_t k = 0; k < nRemoteIn; ++k) acc = red<DT>(op.reduceOp, acc, ld4(rin[k] + b, true));
    st4(out + b, acc, false);
    if constexpr (SendToRemote)
      for (uint32_t k = 0; k < nRemoteOut; ++k) st4(rout[k] + b, acc, true);
  }
}

// handleReduceSend (:446-507): out = src (+) local inputs in listed order; optionally to remotes.
template <int DT, bool ReuseScratch, bool SendToRemote>
__device__ void handleReduceSend(const Op& op, const Ctx& c, uint64_t offset, uint64_t unitSize) {
  if (op.inSize[0] <= offset) return;
  const uint64_t size = umin64(op.inSize[0] - offset, unitSize);
  const uint8_t* src = getBuffer(c, op.inRef[0]) + op.inOff[0] + getOffset<ReuseScratch>(c, op.inRef[0], offset);
  uint8_t* dst = getBuffer(c, op.outRef[0]) + op.outOff[0] + getOffset<ReuseScratch>(c, op.outRef[0], offset);
  const uint32_t nIn = op.nInputs - 1, nOut = op.nOutputs - 1;
  const uint8_t* lin[kMaxBuffersPerOp];
  uint8_t* rout[kMaxBuffersPerOp];
  for (uint32_t k = 0; k < nIn; ++k)
    lin[k] = getBuffer(c, op.inRef[k + 1]) + op.inOff[k + 1] + getOffset<ReuseScratch>(c, op.outRef[k + 1], offset);
  for (uint32_t k = 0; k < nOut; ++k) {
    const uint8_t r = op.outRef[k + 1];
    rout[k] = (uint8_t*)c.h->remotePtr[r] + op.outOff[k + 1] + getOffset<ReuseScratch>(c, c.h->remoteType[r], offset);
  }
  const uint64_t n16 = size / 16;
  for (uint64_t i = threadIdx.x; i < n16; i += blockDim.x) {
    u32x4 acc = ld16(src + i * 16, false);
    for (uint32_t k = 0; k < nIn; ++k) acc = red4<DT>(op.reduceOp, acc, ld16(lin[k] + i * 16, false));
    st16(dst + i * 16, acc, false);
    if constexpr (SendToRemote)
      for (uint32_t k = 0; k < nOut; ++k) st16(rout[k] + i * 16, acc, true);
  }
  for (uint64_t b = n16 * 16 + threadIdx.x * 4; b + 4 <= size; b += (uint64_t)blockDim.x * 4) {
    uint32_t acc = ld4(src + b, false);
    for (uint32_t k = 0; k < nIn; ++k) acc = red<DT>(op.reduceOp, acc, ld4(lin[k] + b, false));
    st4(dst + b, acc, false);
    if constexpr (SendToRemote)
      for (uint32_t k = 0; k < nOut; ++k) st4(rout[k] + b, acc, true);
  }
}

// handlePutPackets (:262-296), memory channels: inputs -> packets in each peer's scratch
template <bool LL16>
__device__ void handlePutPackets(const Op& op, const Ctx& c) {
  const uint8_t* in = getBuffer(c, op.inRef[0]);
  for (uint32_t k = 0; k < op.nOutputs; ++k) {
    uint8_t* dst = (uint8_t*)c.h->remotePtr[op.outRef[k]] + (op.outOff[k] << 1) + c.scratchOffset;
    copyToPackets<LL16>(dst, in + op.inOff[k], op.inSize[k], c.flag);
  }
}

// handleReadPutPackets (:298-337), memory channels: forward local scratch packets to peers
template <bool LL16>
__device__ void handleReadPutPackets(const Op& op, const Ctx& c) {
  using P = Pkt<LL16>;
  const uint64_t n = op.inSize[0] / P::kPayload;
  const uint8_t* pk = c.scratch + c.scratchOffset + (op.inOff[0] << 1);
  for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) {
    uint32_t w0, w1;
    P::read(pk, i, c.flag, w0, w1, c);
    for (uint32_t k = 0; k < op.nOutputs; ++k)
      P::write((uint8_t*)c.h->remotePtr[op.outRef[k]] + c.scratchOffset + (op.outOff[k] << 1), i, w0, w1, c.flag);
  }
}

// handleReduceSendPackets (:339-379): zero, then (+) every packet source in listed order, then
// (+) the local payload; stored locally and, for respkt, sent as packets.
template <int DT, bool LL16, bool SendToRemote>
__device__ void handleReduceSendPackets(const Op& op, const Ctx& c) {
  using P = Pkt<LL16>;
  const uint64_t n = op.inSize[0] / P::kPayload;
  const uint32_t nSrcs = op.nInputs - 1, nDst = op.nOutputs - 1;
  const uint8_t* src = getBuffer(c, op.inRef[0]) + (op.inOff[0] / P::kPayload) * P::kPayload;
  uint8_t* dst = getBuffer(c, op.outRef[0]) + (op.outOff[0] / P::kPayload) * P::kPayload;
  for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) {
    uint32_t a0 = 0, a1 = 0;
    for (uint32_t k = 0; k < nSrcs; ++k) {
      uint32_t w0, w1;
      P::read(c.scratch + c.scratchOffset + 2 * op.inOff[k + 1], i, c.flag, w0, w1, c);
      a0 = red<DT>(op.reduceOp, a0, w0);
      if (LL16) a1 = red<DT>(op.reduceOp, a1, w1);
    }
    uint32_t s0, s1;
    P::loadPayload(src, i, s0, s1);
    a0 = red<DT>(op.reduceOp, a0, s0);
    if (LL16) a1 = red<DT>(op.reduceOp, a1, s1);
    P::storePayload(dst, i, a0, a1);
    if constexpr (SendToRemote)
      for (uint32_t k = 0; k < nDst; ++k)
        P::write((uint8_t*)c.h->remotePtr[op.outRef[k + 1]] + c.scratchOffset + op.outOff[k + 1] * 2, i, a0, a1, c.flag);
  }
}

// handleReduceCopySendPackets (:381-426): as above, plus a local packet copy of the result into
// outputs[1] (recpkt / recspkt).
template <int DT, bool LL16, bool SendToRemote>
__device__ void handleReduceCopySendPackets(const Op& op, const Ctx& c) {
  using P = Pkt<LL16>;
  const uint64_t n = op.inSize[0] / P::kPayload;
  const uint32_t nSrcs = op.nInputs - 1, nDst = op.nOutputs - 2;
  uint8_t* dstPkt = getBuffer(c, op.outRef[1]) + 2 * op.outOff[1];
  const uint8_t* src = getBuffer(c, op.inRef[0]) + (op.inOff[0] / P::kPayload) * P::kPayload;
  uint8_t* dst = getBuffer(c, op.outRef[0]) + (op.outOff[0] / P::kPayload) * P::kPayload;
  for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) {
    uint32_t a0 = 0, a1 = 0;
    for (uint32_t k = 0; k < nSrcs; ++k) {
      uint32_t w0, w1;
      P::read(c.scratch + c.scratchOffset + 2 * op.inOff[k + 1], i, c.flag, w0, w1, c);
      a0 = red<DT>(op.reduceOp, a0, w0);
      if (LL16) a1 = red<DT>(op.reduceOp, a1, w1);
    }
    uint32_t s0, s1;
    P::loadPayload(src, i, s0, s1);
    a0 = red<DT>(op.reduceOp, a0, s0);
    if (LL16) a1 = red<DT>(op.reduceOp, a1, s1);
    P::storePayload(dst, i, a0, a1);
    P::write(dstPkt, i, a0, a1, c.flag);
    if constexpr (SendToRemote)
      for (uint32_t k = 0; k < nDst; ++k)
        P::write((uint8_t*)c.h->remotePtr[op.outRef[k + 2]] + c.scratchOffset + op.outOff[k + 2] * 2, i, a0, a1, c.flag);
  }
}

// handleUnpackPackets (:428-442)
template <bool LL16>
__device__ void handleUnpackPackets(const Op& op, const Ctx& c) {
  using P = Pkt<LL16>;
  const uint64_t n = op.inSize[0] / P::kPayload;
  const uint8_t* pk = c.scratch + c.scratchOffset + (op.inOff[0] << 1);
  uint8_t* out = getBuffer(c, op.outRef[0]) + op.outOff[0];
  for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) {
    uint32_t w0, w1;
    P::read(pk, i, c.flag, w0, w1, c);
    P::storePayload(out, i, w0, w1);
  }
}

// handleCopyPackets (:444-453)
template <bool LL16>
__device__ void handleCopyPackets(const Op& op, const Ctx& c) {
  uint8_t* dst = getBuffer(c, op.outRef[0]) + (op.outOff[0] << 1);
  const uint8_t* src = getBuffer(c, op.inRef[0]) + op.inOff[0];
  copyToPackets<LL16>(dst, src, op.inSize[0], c.flag);
}

// handleSemRelease / handleSemAcquire (:670-684): a counting semaphore per id.  As with
// signal / wait, a release first gathers the workgroup's drained stores and an acquire ends with a
// workgroup barrier, so the semaphore orders whole workgroups.
__device__ void handleSemRelease(const Op& op, const Ctx& c) {
  drain();
  __syncthreads();
  if (threadIdx.x < op.nSems)
    add_release_agent(reinterpret_cast<uint64_t*>(&c.sems[op.semIds[threadIdx.x]].value), 1);
}
__device__ void handleSemAcquire(const Op& op, const Ctx& c) {
  if (threadIdx.x < op.nSems) {
    int64_t* v = &c.sems[op.semIds[threadIdx.x]].value;
    SpinGuard g(c.budget);
    for (;;) {
      int64_t cur = __hip_atomic_load(v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cur > 0 && __hip_atomic_compare_exchange_strong(v, &cur, cur - 1, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT))
        break;
      if (g.expired()) {
        report_error_detail(c.err, kErrSemaphoreTimeout, 0x5E000000u | op.semIds[threadIdx.x], blockIdx.x, 0);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    drain();
  }
  __syncthreads();
}

template <int DT, bool LL16, bool ReuseScratch>
__device__ uint32_t executeOp(const Op* ops, uint32_t i, const Ctx& c, uint64_t offset, uint64_t unitSize);

// handlePipeline (:646-668): the next nOperations operations run nIterations times over
// unitSize-byte windows.
template <int DT, bool LL16, bool ReuseScratch>
__device__ void handlePipeline(const Op* ops, uint32_t i, const Ctx& c) {
  const Op& op = ops[i];
  for (uint32_t it = 0; it < op.nIterations; ++it) {
    const uint64_t offset = (uint64_t)it * op.unitSize;
    for (uint32_t k = 0; k < op.nOperations; ++k) executeOp<DT, LL16, ReuseScratch>(ops, i + 1 + k, c, offset, op.unitSize);
  }
}

// executeDeviceFunction (:700-797); returns the number of plan entries consumed
template <int DT, bool LL16, bool ReuseScratch>
__device__ uint32_t executeOp(const Op* ops, uint32_t i, const Ctx& c, uint64_t offset, uint64_t unitSize) {
  const Op& op = ops[i];
  switch (op.type) {
    case NOP: handleNop(); break;
    case BARRIER: handleBarrier(op, c); break;
    case SIGNAL: handleSignal<false>(op, c); break;
    case WAIT: handleWait<false>(op, c); break;
    case RELAXED_SIGNAL: handleSignal<true>(op, c); break;
    case RELAXED_WAIT: handleWait<true>(op, c); break;
    case PUT:
    case PUT_WITH_SIGNAL:
    case PUT_WITH_SIGNAL_AND_FLUSH: handlePut<ReuseScratch>(op, c, offset, unitSize); break;
    case GET: handleGet<ReuseScratch>(op, c, offset, unitSize); break;
    case COPY: handleCopy<ReuseScratch>(op, c, offset, unitSize); break;
    case READ_REDUCE_SEND: handleReadReduceSend<DT, ReuseScratch, true>(op, c, offset, unitSize); break;
    case READ_REDUCE: handleReadReduceSend<DT, ReuseScratch, false>(op, c, offset, unitSize); break;
    case REDUCE_SEND: handleReduceSend<DT, ReuseScratch, true>(op, c, offset, unitSize); break;
    case REDUCE: handleReduceSend<DT, ReuseScratch, false>(op, c, offset, unitSize); break;
    case PUT_PACKETS: handlePutPackets<LL16>(op, c); break;
    case READ_PUT_PACKETS: handleReadPutPackets<LL16>(op, c); break;
    case REDUCE_SEND_PACKETS: handleReduceSendPackets<DT, LL16, true>(op, c); break;
    case REDUCE_PACKETS: handleReduceSendPackets<DT, LL16, false>(op, c); break;
    case REDUCE_COPY_SEND_PACKETS: handleReduceCopySendPackets<DT, LL16, true>(op, c); break;
    case REDUCE_COPY_PACKETS: handleReduceCopySendPackets<DT, LL16, false>(op, c); break;
    case UNPACK_PACKETS: handleUnpackPackets<LL16>(op, c); break;
    case COPY_PACKETS: handleCopyPackets<LL16>(op, c); break;
    case SEM_ACQUIRE: handleSemAcquire(op, c); break;
    case SEM_RELEASE: handleSemRelease(op, c); break;
    case PIPELINE:
      handlePipeline<DT, LL16, ReuseScratch>(ops, i, c);
      return op.nOperations + 1;
    default: break;  // FLUSH has no memory-channel meaning; multimem ops are rejected at load
  }
  return 1;
}

// executionKernel (:800-842)
template <int DT, bool LL16, bool ReuseScratch>
__global__ void __launch_bounds__(1024) executionKernel(const TbPlan* plans, uint8_t* input, uint8_t* output,
                                                        uint8_t* scratch, uint64_t scratchOffset, uint64_t scratchChunk,
                                                        uint32_t flag, Syncer* syncers, Sem* sems, uint64_t budget,
                                                        uint32_t* err) {
  extern __shared__ uint4 lds[];
  const TbPlan* mine = plans + blockIdx.x;
  const uint32_t nOps = mine->h.nOps;
  const uint32_t words = (uint32_t)((sizeof(TbHeader) + nOps * sizeof(Op)) / 16);
  for (uint32_t k = threadIdx.x; k < words; k += blockDim.x) lds[k] = ((const uint4*)mine)[k];
  __syncthreads();
  const TbPlan* p = (const TbPlan*)lds;
  Ctx c;
  c.input = input;
  c.output = output;
  c.scratch = scratch;
  c.scratchOffset = scratchOffset;
  c.scratchChunk = scratchChunk ? scratchChunk : 1;
  c.flag = flag;
  c.budget = budget;
  c.err = err;
  c.syncers = syncers;
  c.sems = sems;
  c.h = &p->h;
  for (uint32_t i = 0; i < nOps;) i += executeOp<DT, LL16, ReuseScratch>(p->ops, i, c, 0, ~0ull);
}

template <int DT, int OP>
static void launchT(const TbPlan* plans, int nblocks, int nthreads, size_t lds, uint8_t* in, uint8_t* out, uint8_t* scr,
                    uint64_t scrOff, uint64_t scrChunk, uint32_t flag, Syncer* sy, Sem* se, uint64_t budget,
                    uint32_t* err, hipStream_t s, bool ll16, bool reuse) {
  static_assert(OP == kSum || OP == kMin, "");
  if constexpr (OP == kSum) {  // the reduce operation is per plan operation; instantiate by dtype only
    if (ll16 && !reuse)
      hipLaunchKernelGGL((executionKernel<DT, true, false>), dim3(nblocks), dim3(nthreads), lds, s, plans, in, out, scr,
                         scrOff, scrChunk, flag, sy, se, budget, err);
    else if (ll16 && reuse)
      hipLaunchKernelGGL((executionKernel<DT, true, true>), dim3(nblocks), dim3(nthreads), lds, s, plans, in, out, scr,
                         scrOff, scrChunk, flag, sy, se, budget, err);
    else if (!ll16 && !reuse)
      hipLaunchKernelGGL((executionKernel<DT, false, false>), dim3(nblocks), dim3(nthreads), lds, s, plans, in, out, scr,
                         scrOff, scrChunk, flag, sy, se, budget, err);
    else
      hipLaunchKernelGGL((executionKernel<DT, false, true>), dim3(nblocks), dim3(nthreads), lds, s, plans, in, out, scr,
                         scrOff, scrChunk, flag, sy, se, budget, err);
  }
}

}  // namespace exec

// Launch one execution of a device plan (nblocks threadblock plans at `plans`).  Returns 0, 1 on a
// HIP launch error, 4 on invalid arguments, 5 when the grid cannot be resident at once.
int launchExecutionKernel(const exec::TbPlan* plans, int nblocks, int nthreads, size_t ldsBytes, void* input,
                          void* output, void* scratch, uint64_t scratchOffset, uint64_t scratchChunk, uint32_t flag,
                          exec::Syncer* syncers, exec::Sem* sems, int dtype, bool ll16, bool reuseScratch,
                          uint64_t budget, uint32_t* err, hipStream_t s) {
  using namespace exec;
  if (nblocks <= 0 || nthreads <= 0 || nthreads > 1024 || nthreads % 64) return 4;
  // every workgroup of a plan may wait on another: the whole grid must be resident
  if (!grid_coresident(executionKernel<kF16, true, false>, nthreads, nblocks)) return 5;
  // the reduce operation is per plan operation: instantiate by dtype only (FP8 with T == AccumT)
#define MSCCLPP_AMD_EXEC_CASE(DT)                                                                                \
  case DT:                                                                                                        \
    launchT<DT, kSum>(plans, nblocks, nthreads, ldsBytes, (uint8_t*)input, (uint8_t*)output, (uint8_t*)scratch,   \
                      scratchOffset, scratchChunk, flag, syncers, sems, budget, err, s, ll16, reuseScratch);     \
    break;
  switch (dtype) {
    MSCCLPP_AMD_EXEC_CASE(kF16)
    MSCCLPP_AMD_EXEC_CASE(kBF16)
    MSCCLPP_AMD_EXEC_CASE(kF32)
    MSCCLPP_AMD_EXEC_CASE(kI32)
    MSCCLPP_AMD_EXEC_CASE(kU32)
    MSCCLPP_AMD_EXEC_CASE(kE4M3)
    MSCCLPP_AMD_EXEC_CASE(kE5M2)
    MSCCLPP_AMD_EXEC_CASE(kB15)
    MSCCLPP_AMD_EXEC_CASE(kU8)
    default: return 4;
  }
#undef MSCCLPP_AMD_EXEC_CASE
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

}  // namespace mscclpp_amd
