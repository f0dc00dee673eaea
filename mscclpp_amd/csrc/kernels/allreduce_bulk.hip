// Bulk (non-LL) all-pairs AllReduce for large buckets over xGMI.
//
// Reference behaviour: allreduceFullmesh (src/ext/collectives/allreduce/allreduce_fullmesh.cu:24-166,
// the AMD default above 1 MiB, algorithm_selector.cc:129-131) -- a signal-gated reduce-scatter by
// one-sided puts into peer scratch, a local reduction (own slice first, then peers ascending,
// :101-107) and an all-gather by direct writes into every peer's output buffer (:110-113).  The
// ORDER=1 variant sums in ring order x_r, x_{r+1}, ... (allreduceRsAg, allreduce_rsag.cu:85-94),
// the order-stable fp32 sum of BASELINE config 5.
//
// MI355X design:
//  * The whole per-rank slice is exchanged in at most a few passes; scratch is sized for it (HBM is
//    288 GB), so a 48 MiB bucket is one pass with one RS handshake and one AG handshake per block.
//  * Each workgroup owns one channel (its sub-range of every slice) and one semaphore per peer, so
//    workgroups never wait on each other, and every workgroup streams to all 7 peers at once,
//    starting at a different peer (rotation by block index) to keep all 7 xGMI links busy.
//  * Remote stores are 16-byte system-scope write-through buffer stores; each storing wave drains
//    (s_waitcnt vmcnt(0)) before the workgroup barrier, and one lane per peer then signals with a
//    system-scope release atomic add (MemoryDevice2DeviceSemaphore::signal, semaphore_device.hpp:84-90).
//  * Waits are relaxed system-scope polls followed by one system-scope acquire, bounded in time.
#include <cstdlib>

#include "common.hpp"

namespace mscclpp_amd {

struct BulkGeom {
  uint64_t bytes;       // total bytes per rank
  uint64_t slice;       // bytes per rank slice (multiple of 16)
  uint64_t pass;        // slice bytes handled per pass (multiple of 16)
  uint64_t blk;         // bytes of a pass handled by one workgroup (multiple of 16)
  uint32_t npasses;
  uint32_t debug;       // MSCCLPP_AMD_DEBUG_SKIP_HANDSHAKE (bit 0): skip the reduce-scatter handshake.
                        // Diagnostic only -- it makes the result wrong on purpose, so that the
                        // benchmark's bit-exact check can be shown to catch a missing handshake.
  uint64_t* trace;      // phase stamps (mscclppAmdTraceSet) or null
};

__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// All lanes of the block: publish every prior store, then lane p < nranks signals peer p on
// channel `ch`; then lanes wait for the peers' matching signals.
__device__ __forceinline__ void block_handshake(const mscclppAmdRankView& v, int nranks, int rank, uint32_t ch,
                                                uint64_t budget) {
  drain_stores();
  __syncthreads();
  const int p = (int)threadIdx.x;
  if (p < nranks && p != rank) {
    // my token slot inside peer p's token array: [rank][ch]
    uint64_t* remote = v.peerTokens[p] + (uint64_t)rank * kMaxChannels + ch;
    add_release_sys(remote, 1);
    uint64_t* mine = v.tokens + (uint64_t)p * kMaxChannels + ch;
    uint64_t* exp = v.expected + (uint64_t)p * kMaxChannels + ch;
    // the counter lives in ordinary device memory and is touched once per handshake: agent-scope
    // atomics keep it out of any XCD's stale L2 line whichever XCD this block lands on next launch
    const uint64_t want = __hip_atomic_fetch_add(exp, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
    SpinGuard g(budget);
    while (ld_relaxed_sys(mine) < want) {
      __builtin_amdgcn_s_sleep(2);
      if (g.expired()) {
        // detail: channel | peer << 16, rank, tokens seen (low 16 bits) | wanted (low 16 bits) << 16
        report_error_detail(v.err, kErrSemaphoreTimeout, ch | ((uint32_t)p << 16), (uint32_t)rank,
                            ((uint32_t)ld_relaxed_sys(mine) & 0xffffu) | ((uint32_t)want << 16));
        break;
      }
    }
    acquire_sys();  // the invalidate completes before the barrier
  }
  __syncthreads();
}

// MODE 0: AllReduce.  MODE 1: ReduceScatter (input n*slice, output = my reduced slice; no
// all-gather).  MODE 2: AllGather (input = my slice, output n*slice; no reduce-scatter, no sum).
template <int DT, int OP, int NV, int ORDER, int MODE>
__global__ void __launch_bounds__(512) allreduceBulkKernel(Views<NV> views, BulkGeom g, int nranks, uint64_t budget) {
  const mscclppAmdRankView& v = views.v[NV == 1 ? 0 : blockIdx.y];
  const int rank = v.rank;
  const uint32_t T = blockDim.x, tid = threadIdx.x, b = blockIdx.x;
  const uint8_t* in = (const uint8_t*)v.input;
  uint8_t* out = (uint8_t*)v.output;
  uint8_t* scr = (uint8_t*)v.scratch;
  constexpr int U = 8;  // units per lane per step (128 B in flight per lane in the put phase)
  trace_stamp(g.trace, 0);

  // AllGather writes straight into the peers' outputs: first make sure every peer's kernel is
  // running, i.e. all earlier work on the peer's stream (which may still write that memory, e.g. a
  // framework's freed-and-reused allocation) is done.  AllReduce / ReduceScatter reach the peers'
  // outputs only after their reduce-scatter handshake, which already orders this.
  if constexpr (MODE == 2) block_handshake(v, nranks, rank, b, budget);

  for (uint32_t ps = 0; ps < g.npasses; ++ps) {
    const uint64_t pOff = (uint64_t)ps * g.pass;          // offset inside a slice
    const uint64_t bOff = pOff + (uint64_t)b * g.blk;     // this block's sub-range start in a slice
    uint64_t bLen = 0;
    if ((uint64_t)b * g.blk < g.pass && bOff < g.slice) {
      bLen = g.blk;
      if (bOff + bLen > pOff + g.pass) bLen = pOff + g.pass - bOff;
      if (bOff + bLen > g.slice) bLen = g.slice - bOff;
    }
    const uint32_t nUnits = (uint32_t)((bLen + 15) / 16);

    if constexpr (MODE != 2) {
      // ---- reduce-scatter: put my copy of every peer's slice sub-range into that peer's scratch
      if (nUnits) {
#pragma unroll 1
        for (int i = 0; i < nranks - 1; ++i) {
          // rotate the first peer by block index so concurrent blocks start on different links
          const int k = (i + (int)b) % (nranks - 1);
          const int q = k < rank ? k : k + 1;
          const uint64_t srcOff = (uint64_t)q * g.slice + bOff;
          const auto rsrc = make_rsrc(in + srcOff);
          const uint64_t valid = g.bytes > srcOff ? g.bytes - srcOff : 0;
          const auto rq = make_rsrc((uint8_t*)v.peerScratch[q] + (uint64_t)rank * g.pass + (bOff - pOff));
          for (uint32_t u0 = tid; u0 < nUnits; u0 += T * U) {
            u32x4 w[U];
#pragma unroll
            for (int k2 = 0; k2 < U; ++k2) {
              const uint32_t u = u0 + k2 * T;
              if (u < nUnits)
                w[k2] = load_payload<kNonTemporal>(rsrc, in + srcOff, (uint64_t)u * 16, clamp_valid(valid, (uint64_t)u * 16, 16));
            }
#pragma unroll
            for (int k2 = 0; k2 < U; ++k2) {
              const uint32_t u = u0 + k2 * T;
              if (u < nUnits) store16<kSystem>(rq, u * 16u, w[k2]);
            }
          }
        }
      }
      trace_stamp(g.trace, 1);
      if (!(g.debug & 1u)) block_handshake(v, nranks, rank, b, budget);
      trace_stamp(g.trace, 2);
    }

    // ---- my slice sub-range: reduce (AR, RS), write locally, and (AR, AG) into every peer's output
    if (nUnits) {
      const uint64_t myOff = (uint64_t)rank * g.slice + bOff;
      const uint8_t* myIn = MODE == 2 ? in + bOff : in + myOff;
      uint8_t* myOut = MODE == 1 ? out + bOff : out + myOff;
      const uint64_t valid = MODE == 2 ? g.slice - bOff : (g.bytes > myOff ? g.bytes - myOff : 0);
      const auto rin = make_rsrc(myIn);
      const auto rout = make_rsrc(myOut);
      const auto rscr = make_rsrc(scr + (bOff - pOff));
      for (uint32_t u = tid; u < nUnits; u += T) {
        const uint32_t vb = clamp_valid(valid, (uint64_t)u * 16, 16);
        u32x4 acc = load_payload<kNonTemporal>(rin, myIn, (uint64_t)u * 16, vb);
        if constexpr (MODE != 2) {
          u32x4 w[kMaxRanks];
#pragma unroll
          for (int k = 1; k < kMaxRanks; ++k) {
            if (k < nranks) {
              const int src = ORDER == 0 ? (k - 1 < rank ? k - 1 : k) : (rank + k) % nranks;
              w[k] = load16<kSystem>(rscr, (uint32_t)((uint64_t)src * g.pass) + u * 16u);
            }
          }
          if constexpr (AccWord<DT, OP>::kWide) {
            // calVectorAccum<T, AccumT> (allreduce_fullmesh.cu:102-108, allreduce_rsag.cu:88-95)
            Accum<DT, OP, 4> sum(acc);
#pragma unroll
            for (int k = 1; k < kMaxRanks; ++k)
              if (k < nranks) sum.add(w[k]);
            acc = sum.template get<u32x4>();
          } else {
#pragma unroll
            for (int k = 1; k < kMaxRanks; ++k)
              if (k < nranks) acc = reduce4<DT, OP>(acc, w[k]);
          }
        }
        store_payload<kPlain>(rout, myOut, (uint64_t)u * 16, acc, vb);
        if constexpr (MODE != 1) {
#pragma unroll 1
          for (int i = 0; i < nranks - 1; ++i) {
            const int k = (i + (int)b) % (nranks - 1);
            const int q = k < rank ? k : k + 1;
            uint8_t* po = (uint8_t*)v.peerOutput[q] + myOff;
            if (vb >= 16)
              store16<kSystem>(make_rsrc(po), u * 16u, acc);
            else
              store_tail(po + (uint64_t)u * 16, acc, vb);
          }
        }
      }
    }
    trace_stamp(g.trace, 3);
    block_handshake(v, nranks, rank, b, budget);
  }
  trace_stamp(g.trace, 4);
}

// Zero-copy RS+AG (allreduceRsAgZeroCopy, allreduce_rsag_zero_copy.cu:41-112): no scratch.  Each
// rank reads its own slice straight out of every peer's input buffer over xGMI, sums in ring order
// (own, r+1, r+2, ...; :90-96), and writes the result into its own output and every peer's output
// (:101-106).  Per channel (= workgroup) one handshake at entry -- the peers' inputs are ready and
// their previous call no longer reads mine or writes my output -- and one at exit, after every
// wave has drained its remote stores, so each output is complete when the kernel ends.  xGMI bytes
// per rank and direction equal fullmesh's (2*(n-1)/n*S); HBM traffic drops by the scratch
// round trip.
template <int DT, int OP, int NV>
__global__ void __launch_bounds__(512) allreduceZeroCopyKernel(Views<NV> views, BulkGeom g, int nranks, uint64_t budget) {
  const mscclppAmdRankView& v = views.v[NV == 1 ? 0 : blockIdx.y];
  const int rank = v.rank;
  const uint32_t T = blockDim.x, tid = threadIdx.x, b = blockIdx.x;
  const uint64_t bOff = (uint64_t)b * g.blk;
  uint64_t bLen = 0;
  if (bOff < g.slice) bLen = (bOff + g.blk > g.slice) ? g.slice - bOff : g.blk;
  const uint32_t nUnits = (uint32_t)((bLen + 15) / 16);
  trace_stamp(g.trace, 0);
  block_handshake(v, nranks, rank, b, budget);
  trace_stamp(g.trace, 1);
  const uint64_t myOff = (uint64_t)rank * g.slice + bOff;
  if (nUnits && myOff < g.bytes) {
    const uint64_t valid = g.bytes - myOff;
    const uint8_t* myIn = (const uint8_t*)v.input + myOff;
    uint8_t* myOut = (uint8_t*)v.output + myOff;
    const auto rin = make_rsrc(myIn);
    const auto rout = make_rsrc(myOut);
    for (uint32_t u = tid; u < nUnits; u += T) {
      const uint32_t vb = clamp_valid(valid, (uint64_t)u * 16, 16);
      if (vb == 0) break;
      const u32x4 own = load_payload<kNonTemporal>(rin, myIn, (uint64_t)u * 16, vb);
      u32x4 w[kMaxRanks];
#pragma unroll
      for (int k = 1; k < kMaxRanks; ++k) {
        if (k < nranks) {
          const uint8_t* pin = (const uint8_t*)v.peerInput[(rank + k) % nranks] + myOff;
          w[k] = vb >= 16 ? load16<kSystem>(make_rsrc(pin), u * 16u) : load_tail(pin + (uint64_t)u * 16, vb);
        }
      }
      u32x4 acc;
      if constexpr (AccWord<DT, OP>::kWide) {
        Accum<DT, OP, 4> sum(own);
#pragma unroll
        for (int k = 1; k < kMaxRanks; ++k)
          if (k < nranks) sum.add(w[k]);
        acc = sum.template get<u32x4>();
      } else {
        acc = own;
#pragma unroll
        for (int k = 1; k < kMaxRanks; ++k)
          if (k < nranks) acc = reduce4<DT, OP>(acc, w[k]);
      }
      store_payload<kPlain>(rout, myOut, (uint64_t)u * 16, acc, vb);
#pragma unroll 1
      for (int k = 1; k < nranks; ++k) {
        uint8_t* po = (uint8_t*)v.peerOutput[(rank + k) % nranks] + myOff;
        if (vb >= 16)
          store16<kSystem>(make_rsrc(po), u * 16u, acc);
        else
          store_tail(po + (uint64_t)u * 16, acc, vb);
      }
    }
  }
  trace_stamp(g.trace, 2);
  block_handshake(v, nranks, rank, b, budget);
  trace_stamp(g.trace, 3);
}

// mscclpp-test allreduce5, AMD branch (test/mscclpp-test/allreduce_test.cu:959-970 ->
// localReduceScatterMem3 :375-435, localRingAllGatherMem2 :586-617): in place on the user buffer,
// no scratch.  Reduce-scatter: rank r adds chunk r of every peer's buffer (remote reads, channel
// order (i + r) % nPeers, :402-404) into its own chunk r; all-gather: rank r gets chunk q out of
// rank q's buffer (same channel order, :604-608).  The reference gates each phase with one
// signal/wait per peer plus a grid-wide DeviceSyncer; here each workgroup owns the same sub-range
// of every chunk in both phases and handshakes only with the peers' workgroup of the same index --
// at entry, between the phases (a peer overwrites its copy of my chunk only in its all-gather,
// after I have read it) and at exit (peers have finished reading my buffer when my kernel ends).
template <int DT, int OP, int NV>
__global__ void __launch_bounds__(512) allreduceTestK5Kernel(Views<NV> views, BulkGeom g, int nranks, uint64_t budget) {
  const mscclppAmdRankView& v = views.v[NV == 1 ? 0 : blockIdx.y];
  const int rank = v.rank;
  const int nPeers = nranks - 1;
  const uint32_t T = blockDim.x, tid = threadIdx.x, b = blockIdx.x;
  const uint64_t bOff = (uint64_t)b * g.blk;
  uint64_t bLen = 0;
  if (bOff < g.slice) bLen = (bOff + g.blk > g.slice) ? g.slice - bOff : g.blk;
  const uint32_t nUnits = (uint32_t)(bLen / 16);  // the host keeps chunks a multiple of 16 bytes
  uint8_t* buf = (uint8_t*)v.output;
  auto peerOf = [&](int i) {  // channel (i + rank) % nPeers -> its rank
    const int c = (i + rank) % nPeers;
    return c < rank ? c : c + 1;
  };
  block_handshake(v, nranks, rank, b, budget);
  {
    const uint64_t off = (uint64_t)rank * g.slice + bOff;
    const auto rb = make_rsrc(buf + off);
    for (uint32_t u = tid; u < nUnits; u += T) {
      u32x4 w[kMaxRanks];
#pragma unroll
      for (int i = 0; i < kMaxRanks - 1; ++i)
        if (i < nPeers) w[i] = load16<kSystem>(make_rsrc((const uint8_t*)v.peerOutput[peerOf(i)] + off), u * 16u);
      u32x4 acc = load16<kPlain>(rb, u * 16u);
#pragma unroll
      for (int i = 0; i < kMaxRanks - 1; ++i)
        if (i < nPeers) acc = reduce4<DT, OP>(acc, w[i]);
      store16<kPlain>(rb, u * 16u, acc);
    }
  }
  block_handshake(v, nranks, rank, b, budget);
#pragma unroll 1
  for (int i = 0; i < nPeers; ++i) {
    const int q = peerOf(i);
    const uint64_t off = (uint64_t)q * g.slice + bOff;
    const auto rsrc = make_rsrc((const uint8_t*)v.peerOutput[q] + off);
    const auto rdst = make_rsrc(buf + off);
    for (uint32_t u = tid; u < nUnits; u += T) store16<kPlain>(rdst, u * 16u, load16<kSystem>(rsrc, u * 16u));
  }
  block_handshake(v, nranks, rank, b, budget);
}

// ncclBroadcast (nccl.cc:549-605; the reference runs it through its algorithm collection or falls
// back to NCCL): a zero-copy pull from the root.  Each workgroup owns one sub-range.  Entry
// handshake: the root's send buffer is final (its producer ran earlier on the root's stream) and
// every reader's previous use of its receive buffer is over.  Non-roots then read the root's send
// buffer over xGMI (system-scope 16-byte loads) and store into their own receive buffer; the root
// copies send -> recv when out of place.  Exit handshake: every reader is done with the root's
// buffer before any rank's kernel ends, so the root may overwrite it in its next stream operation.
template <int NV, int U>
__global__ void __launch_bounds__(512) broadcastKernel(Views<NV> views, uint64_t bytes, uint64_t blk, int nranks,
                                                       int root, uint64_t budget) {
  const mscclppAmdRankView& v = views.v[NV == 1 ? 0 : blockIdx.y];
  const int rank = v.rank;
  const uint32_t T = blockDim.x, tid = threadIdx.x, b = blockIdx.x;
  const uint64_t bOff = (uint64_t)b * blk;
  block_handshake(v, nranks, rank, b, budget);
  if (bOff < bytes) {
    const uint64_t len = bytes - bOff < blk ? bytes - bOff : blk;
    const uint8_t* src = (rank == root ? (const uint8_t*)v.input : (const uint8_t*)v.peerInput[root]) + bOff;
    uint8_t* dst = (uint8_t*)v.output + bOff;
    if (src != dst) {
      const auto rs = make_rsrc(src);
      const auto rd = make_rsrc(dst);
      const uint32_t nUnits = (uint32_t)((len + 15) / 16);
      for (uint32_t u0 = tid; u0 < nUnits; u0 += T * U) {
        u32x4 w[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
          const uint32_t u = u0 + k * T;
          const uint32_t vb = u < nUnits ? clamp_valid(len, (uint64_t)u * 16, 16) : 0;
          if (vb >= 16)
            w[k] = load16<kSystem>(rs, u * 16u);
          else if (vb)
            w[k] = load_tail(src + (uint64_t)u * 16, vb);
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
          const uint32_t u = u0 + k * T;
          if (u < nUnits) store_payload<kPlain>(rd, dst, (uint64_t)u * 16, w[k], clamp_valid(len, (uint64_t)u * 16, 16));
        }
      }
    }
  }
  block_handshake(v, nranks, rank, b, budget);
}

// Pipelined RS+AG (allreduceRsAgPipeline, allreduce_rsag_pipeline.cu:85-222).  Three roles run at
// once in one launch: P = R/2 put workgroups, R reduce workgroups, V = R/2 recv workgroups.  One
// iteration covers n slots of C = R * T * 4 units (16 B) each; slot q holds the units rank q owns.
//   put p    : waits for a free scratch stage (credit from recv p, pipeline depth D), writes its
//              share of every peer's slot into that peer's scratch RS region (remote 16-B stores),
//              drains, releases reduce 2p and 2p+1.
//   reduce b : waits for put b/2, handshakes with the peers' reduce b (their puts into my RS region
//              are done), sums own + peers in ring order (own, r+1, ...; the reference's
//              calVector(data, tmp), :160-166), stores the result locally and into every peer's AG
//              region, drains, releases recv b/2.
//   recv v   : waits for reduce 2v and 2v+1, handshakes with the peers' recv v (their reduced
//              slots are in my AG region), copies them into the output, releases the credit.
// Every remote store lands in communicator-owned scratch (nothing written into peers' user
// buffers), and the iterations overlap.  Intra-launch counters live in v.pipeSems: [0, 256)
// recv->put credits, [256, 512) put->reduce, [512, 768) reduce->recv, [768] workgroups done.  They
// are zero when a launch starts: zeroed once at allocation, and the last workgroup of every launch
// to finish puts them back to zero (a stream-ordered memset before each launch did the same in
// eager mode, but in a replayed HIP graph the kernel read the previous replay's counters -- every
// replay after the first came back with stale data, tests/test_graph_capture_gpu.py).
struct PipeGeom {
  uint64_t bytes;   // buffer bytes
  uint64_t C;       // units per slot and iteration
  uint32_t nIters;  // iterations
  uint32_t D;       // pipeline depth (stages in the scratch)
  uint32_t R;       // reduce workgroups (P = V = R / 2)
  uint32_t pad;
};

__device__ __forceinline__ void sem_release(uint64_t* c) {
  drain_stores();
  __syncthreads();
  if (threadIdx.x == 0) add_release_agent(c, 1);
}

// End of a pipeline workgroup: count it done; the last of the launch's `total` workgroups (every
// other one has made its last counter access before counting itself) zeroes the counters for the
// next launch.
__device__ __forceinline__ void pipe_done(uint64_t* sems, uint32_t R, uint32_t total) {
  __syncthreads();
  if (threadIdx.x == 0) {
    if (add_release_agent(sems + 768, 1) == total - 1) {
      acquire_agent();
      for (uint32_t i = 0; i < R / 2; ++i) __hip_atomic_store(sems + i, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (uint32_t i = 0; i < R; ++i) {
        __hip_atomic_store(sems + 256 + i, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(sems + 512 + i, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __hip_atomic_store(sems + 768, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__device__ __forceinline__ void sem_acquire(uint64_t* c, uint64_t target, uint64_t budget, uint32_t* err) {
  if (threadIdx.x == 0) {
    SpinGuard g(budget);
    while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (g.expired()) {
        report_error(err, kErrSemaphoreTimeout);
        break;
      }
    }
    acquire_agent();
  }
  __syncthreads();
}

template <int DT, int OP, int NV>
__global__ void __launch_bounds__(512) allreduceRsAgPipelineKernel(Views<NV> views, PipeGeom g, int nranks,
                                                                   uint64_t budget) {
  const mscclppAmdRankView& v = views.v[NV == 1 ? 0 : blockIdx.y];
  const int rank = v.rank;
  const uint32_t T = blockDim.x, tid = threadIdx.x, bid = blockIdx.x;
  const uint32_t P = g.R / 2;
  const uint64_t C = g.C, nC = (uint64_t)nranks * C;
  uint64_t* credit = v.pipeSems;
  uint64_t* toReduce = v.pipeSems + 256;
  uint64_t* toRecv = v.pipeSems + 512;
  const uint8_t* in = (const uint8_t*)v.input;
  uint8_t* out = (uint8_t*)v.output;
  uint8_t* scr = (uint8_t*)v.scratch;
  // byte offset of (iteration, slot q) in the buffer, and of (stage, region, slot q) in the scratch
  auto bufOff = [&](uint32_t it, int q) { return ((uint64_t)it * nC + (uint64_t)q * C) * 16; };
  auto scrOff = [&](uint32_t it, int region, int q) {
    return ((uint64_t)(it % g.D) * 2 * nC + (uint64_t)region * nC + (uint64_t)q * C) * 16;
  };
  if (bid < P) {  // ---- put
    const uint32_t p = bid;
    for (uint32_t it = 0; it < g.nIters; ++it) {
      if (it >= g.D) sem_acquire(&credit[p], it - g.D + 1, budget, v.err);
#pragma unroll 1
      for (int k = 1; k < nranks; ++k) {
        const int q = (rank + k) % nranks;  // (rank + peer + 1) % n (:112-113)
        const uint64_t so = bufOff(it, q);
        const auto rs = make_rsrc(in + so);
        const auto rd = make_rsrc((uint8_t*)v.peerScratch[q] + scrOff(it, 0, rank));
        u32x4 w[8];
#pragma unroll
        for (int st = 0; st < 8; ++st) {
          const uint32_t pos = p * T + tid + st * T * P;
          const uint32_t vb = clamp_valid(g.bytes, so + (uint64_t)pos * 16, 16);
          w[st] = vb >= 16 ? load16<kNonTemporal>(rs, pos * 16u) : vb ? load_tail(in + so + (uint64_t)pos * 16, vb) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int st = 0; st < 8; ++st) {
          const uint32_t pos = p * T + tid + st * T * P;
          if (so + (uint64_t)pos * 16 < g.bytes) store16<kSystem>(rd, pos * 16u, w[st]);
        }
      }
      sem_release(&toReduce[2 * p]);
      // (thread 0's release above already wrote the L2 back and waited: a relaxed add stays behind it)
      if (tid == 0) __hip_atomic_fetch_add(&toReduce[2 * p + 1], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    pipe_done(v.pipeSems, g.R, 2 * g.R);
  } else if (bid < P + g.R) {  // ---- reduce
    const uint32_t b = bid - P, p = b / 2, sub = b % 2;
    for (uint32_t it = 0; it < g.nIters; ++it) {
      sem_acquire(&toReduce[b], it + 1, budget, v.err);
      block_handshake(v, nranks, rank, b, budget);  // peers' puts into my RS region (these units) done
      const uint64_t mo = bufOff(it, rank);
      const auto rin = make_rsrc(in + mo);
      const auto rout = make_rsrc(out + mo);
      const auto rrs = make_rsrc(scr + scrOff(it, 0, 0));
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        const uint32_t pos = p * T + tid + (sub * 4 + st) * T * P;
        const uint32_t vb = clamp_valid(g.bytes, mo + (uint64_t)pos * 16, 16);
        if (vb == 0) continue;
        u32x4 acc = load_payload<kNonTemporal>(rin, in + mo, (uint64_t)pos * 16, vb);
#pragma unroll
        for (int k = 1; k < kMaxRanks; ++k) {
          if (k < nranks) {
            const int q = (rank + k) % nranks;
            const u32x4 d = load16<kSystem>(rrs, (uint32_t)((uint64_t)q * C * 16) + pos * 16u);
            acc = reduce4<DT, OP>(d, acc);  // calVector<T, OpType>(data, tmp)
          }
        }
        store_payload<kPlain>(rout, out + mo, (uint64_t)pos * 16, acc, vb);
#pragma unroll 1
        for (int k = 1; k < nranks; ++k) {
          const int q = (rank + k) % nranks;
          store16<kSystem>(make_rsrc((uint8_t*)v.peerScratch[q] + scrOff(it, 1, rank)), pos * 16u, acc);
        }
      }
      sem_release(&toRecv[b]);
    }
    pipe_done(v.pipeSems, g.R, 2 * g.R);
  } else {  // ---- recv
    const uint32_t r = bid - P - g.R;
    for (uint32_t it = 0; it < g.nIters; ++it) {
      sem_acquire(&toRecv[2 * r], it + 1, budget, v.err);
      sem_acquire(&toRecv[2 * r + 1], it + 1, budget, v.err);
      block_handshake(v, nranks, rank, g.R + r, budget);  // peers' reduced slots are in my AG region
#pragma unroll 1
      for (int k = 1; k < nranks; ++k) {
        const int q = (rank + k) % nranks;
        const uint64_t oo = bufOff(it, q);
        const auto rag = make_rsrc(scr + scrOff(it, 1, q));
        const auto rout = make_rsrc(out + oo);
        u32x4 w[8];
#pragma unroll
        for (int st = 0; st < 8; ++st) {
          const uint32_t pos = r * T + tid + st * T * P;
          if (oo + (uint64_t)pos * 16 < g.bytes) w[st] = load16<kSystem>(rag, pos * 16u);
        }
#pragma unroll
        for (int st = 0; st < 8; ++st) {
          const uint32_t pos = r * T + tid + st * T * P;
          const uint32_t vb = clamp_valid(g.bytes, oo + (uint64_t)pos * 16, 16);
          if (vb) store_payload<kPlain>(rout, out + oo, (uint64_t)pos * 16, w[st], vb);
        }
      }
      sem_release(&credit[r]);
    }
    // Exit: every peer's recv v has copied my reduced slots out of ITS scratch before my kernel
    // ends.  Without this a collective issued next on this communicator (fullmesh / reduce-scatter
    // put into the peers' scratch with no entry handshake) could overwrite a peer's AG region while
    // that peer is still copying it.  The peers' reduce workgroups are done too: their recv waited
    // for them.  Same channel as the entry handshakes, so every rank's counters stay in step.
    block_handshake(v, nranks, rank, g.R + r, budget);
    pipe_done(v.pipeSems, g.R, 2 * g.R);
  }
}

static thread_local int g_launch_status = 0;

// Each workgroup addresses its sub-range of a buffer from one buffer resource (32-bit offsets): a
// launch whose per-workgroup range would exceed that is refused (ncclInvalidUsage) -- more
// workgroups carry it (every default shape does up to hundreds of GiB).
constexpr uint64_t kBlkOffsetLimit = 0xFFFFFFFFull - 64;

size_t bulkScratchRequired(int nranks, size_t bytes, size_t maxScratch, BulkGeom* out, int nblocks) {
  BulkGeom g{};
  g.trace = g_mscclppAmdTrace;
  g.bytes = bytes;
  const uint64_t per = (bytes + nranks - 1) / nranks;
  g.slice = (per + 15) & ~15ull;
  // largest pass whose n regions fit the scratch budget, and the 32-bit offsets of the one buffer
  // resource the reduce step reads all n regions through (source q at q * pass)
  uint64_t pass = g.slice;
  uint64_t cap = maxScratch / (uint64_t)nranks;
  const uint64_t cap32 = (0xFFFFFFFFull - 64) / (uint64_t)nranks;
  if (cap > cap32) cap = cap32;
  if (pass > cap) pass = cap / ((uint64_t)16 * nblocks) * ((uint64_t)16 * nblocks);
  if (pass == 0) return 0;
  g.pass = pass;
  g.npasses = (uint32_t)((g.slice + pass - 1) / pass);
  g.blk = ((pass + nblocks - 1) / nblocks + 15) & ~15ull;
  if (out) *out = g;
  return (size_t)(nranks * pass);
}

template <int DT, int OP, int NV, int ORDER>
static void launchBulkT(const Views<NV>& vw, int nviews, const BulkGeom& g, int nranks, int nblocks, int nthreads, uint64_t budget,
                        hipStream_t s, int mode) {
  if (!grid_coresident(allreduceBulkKernel<DT, OP, NV, ORDER, 0>, nthreads, (long)nblocks * nviews)) {
    g_launch_status = 5;  // ncclInvalidUsage: the grid cannot be resident at once: its handshakes would deadlock
    return;
  }
  if (mode == 0)
    hipLaunchKernelGGL((allreduceBulkKernel<DT, OP, NV, ORDER, 0>), dim3(nblocks, nviews), dim3(nthreads), 0, s, vw, g,
                       nranks, budget);
  else if (mode == 1)
    hipLaunchKernelGGL((allreduceBulkKernel<DT, OP, NV, ORDER, 1>), dim3(nblocks, nviews), dim3(nthreads), 0, s, vw, g,
                       nranks, budget);
  else if constexpr (ORDER == 0 && OP == kSum && (DT == kF16 || DT == kF32))
    // AllGather moves bytes only: one instantiation per element width is enough
    hipLaunchKernelGGL((allreduceBulkKernel<DT, OP, NV, ORDER, 2>), dim3(nblocks, nviews), dim3(nthreads), 0, s, vw, g,
                       nranks, budget);
}

template <int DT, int OP>
static void launchBulk(const mscclppAmdRankView* views, int nviews, const BulkGeom& g, int nranks, int nblocks,
                       int nthreads, uint64_t budget, hipStream_t s, int order, int mode) {
  if (nviews == 1) {
    Views<1> vw;
    vw.v[0] = views[0];
    if (order == 0)
      launchBulkT<DT, OP, 1, 0>(vw, nviews, g, nranks, nblocks, nthreads, budget, s, mode);
    else
      launchBulkT<DT, OP, 1, 1>(vw, nviews, g, nranks, nblocks, nthreads, budget, s, mode);
  } else {
    Views<kMaxRanks> vw{};
    for (int i = 0; i < nviews; ++i) vw.v[i] = views[i];
    if (order == 0)
      launchBulkT<DT, OP, kMaxRanks, 0>(vw, nviews, g, nranks, nblocks, nthreads, budget, s, mode);
    else
      launchBulkT<DT, OP, kMaxRanks, 1>(vw, nviews, g, nranks, nblocks, nthreads, budget, s, mode);
  }
}

// mode 0 AllReduce (bytes = whole buffer), 1 ReduceScatter / 2 AllGather (bytes = n * block, block % 16 == 0)
template <int DT, int OP, int NV>
static void launchZeroCopyT(const Views<NV>& vw, int nviews, const BulkGeom& g, int nranks, int nblocks, int nthreads,
                            uint64_t budget, hipStream_t s) {
  if (!grid_coresident(allreduceZeroCopyKernel<DT, OP, NV>, nthreads, (long)nblocks * nviews)) {
    g_launch_status = 5;  // ncclInvalidUsage: handshakes of a non-resident grid would deadlock
    return;
  }
  hipLaunchKernelGGL((allreduceZeroCopyKernel<DT, OP, NV>), dim3(nblocks, nviews), dim3(nthreads), 0, s, vw, g, nranks,
                     budget);
}

template <int DT, int OP>
static void launchZeroCopy(const mscclppAmdRankView* views, int nviews, const BulkGeom& g, int nranks, int nblocks,
                           int nthreads, uint64_t budget, hipStream_t s) {
  if (nviews == 1) {
    Views<1> vw;
    vw.v[0] = views[0];
    launchZeroCopyT<DT, OP, 1>(vw, nviews, g, nranks, nblocks, nthreads, budget, s);
  } else {
    Views<kMaxRanks> vw{};
    for (int i = 0; i < nviews; ++i) vw.v[i] = views[i];
    launchZeroCopyT<DT, OP, kMaxRanks>(vw, nviews, g, nranks, nblocks, nthreads, budget, s);
  }
}

int launchCollectiveBulk(int mode, int algo, const mscclppAmdRankView* views, int nviews, int nranks, size_t bytes,
                         int dtype, int op, int nblocks, int nthreads, uint64_t budget, hipStream_t s) {
  if (nblocks <= 0) nblocks = 64;
  if (nthreads <= 0) nthreads = 512;
  if (nblocks > kMaxChannels || nthreads > 512 || nthreads % 64 || nthreads < 64) return 4;
  if (algo == MSCCLPP_AMD_ALGO_TEST_K5) {
    // (the harness launches 24 x 1024, allreduce_test.cu:1126-1129; here the channel defaults apply)
    if (mode != 0 || (dtype != kI32 && dtype != kU32)) return 4;
    if (bytes % ((size_t)16 * nranks)) return 5;  // chunks of whole 16-byte units (reference: 4 * worldSize)
    for (int i = 0; i < nviews; ++i)
      if (views[i].input != views[i].output) return 5;  // allreduce5 runs in place (isInPlace, :1262-1264)
    BulkGeom g{};
    g.trace = g_mscclppAmdTrace;
    g.bytes = bytes;
    g.slice = bytes / nranks;
    g.pass = g.slice;
    g.npasses = 1;
    g.blk = ((g.slice + nblocks - 1) / nblocks + 15) & ~15ull;
    if (g.blk > kBlkOffsetLimit) return 5;  // more workgroups needed: one workgroup's range is one descriptor
    g_launch_status = 0;
    auto go = [&](auto kern) {
      if (!grid_coresident(kern, nthreads, (long)nblocks * nviews)) {
        g_launch_status = 5;
        return;
      }
      if (nviews == 1) {
        Views<1> vw;
        vw.v[0] = views[0];
        hipLaunchKernelGGL(kern, dim3(nblocks, nviews), dim3(nthreads), 0, s, vw, g, nranks, budget);
      }
    };
    auto goN = [&](auto kern) {
      if (!grid_coresident(kern, nthreads, (long)nblocks * nviews)) {
        g_launch_status = 5;
        return;
      }
      Views<kMaxRanks> vw{};
      for (int i = 0; i < nviews; ++i) vw.v[i] = views[i];
      hipLaunchKernelGGL(kern, dim3(nblocks, nviews), dim3(nthreads), 0, s, vw, g, nranks, budget);
    };
    const bool u32 = dtype == kU32, mn = op == kMin;
    if (nviews == 1) {
      if (u32) mn ? go(allreduceTestK5Kernel<kU32, kMin, 1>) : go(allreduceTestK5Kernel<kU32, kSum, 1>);
      else mn ? go(allreduceTestK5Kernel<kI32, kMin, 1>) : go(allreduceTestK5Kernel<kI32, kSum, 1>);
    } else {
      if (u32) mn ? goN(allreduceTestK5Kernel<kU32, kMin, kMaxRanks>) : goN(allreduceTestK5Kernel<kU32, kSum, kMaxRanks>);
      else mn ? goN(allreduceTestK5Kernel<kI32, kMin, kMaxRanks>) : goN(allreduceTestK5Kernel<kI32, kSum, kMaxRanks>);
    }
    if (g_launch_status) return g_launch_status;
    return hipGetLastError() == hipSuccess ? 0 : 1;
  }
  if (algo == MSCCLPP_AMD_ALGO_RSAG_ZC) {
    if (mode != 0) return 4;
    BulkGeom g{};
    g.trace = g_mscclppAmdTrace;
    g.bytes = bytes;
    g.slice = ((bytes + nranks - 1) / nranks + 15) & ~15ull;
    g.pass = g.slice;
    g.npasses = 1;
    g.blk = ((g.slice + nblocks - 1) / nblocks + 15) & ~15ull;
    if (g.blk > kBlkOffsetLimit) return 5;
    g_launch_status = 0;
    MSCCLPP_AMD_DISPATCH_ALL(dtype, op, launchZeroCopy, views, nviews, g, nranks, nblocks, nthreads, budget, s);
    if (g_launch_status) return g_launch_status;
    return hipGetLastError() == hipSuccess ? 0 : 1;
  }
  if (mode != 0 && (bytes % ((size_t)16 * nranks))) return 5;
  BulkGeom g{};
  g.trace = g_mscclppAmdTrace;
  if (!bulkScratchRequired(nranks, bytes, views[0].scratchBytes, &g, nblocks)) return 5;
  const int order = (algo == MSCCLPP_AMD_ALGO_RSAG && mode != 2) ? 1 : 0;
  static const uint32_t debug = [] {
    const char* e = std::getenv("MSCCLPP_AMD_DEBUG_SKIP_HANDSHAKE");
    return (e && *e == '1') ? 1u : 0u;
  }();
  g.debug = mode == 0 ? debug : 0u;
  if (mode == 2) {  // byte movement only: map to the f16 or f32 instantiation by element width
    dtype = elem_bytes(dtype) == 2 ? kF16 : kF32;
    op = kSum;
  }
  g_launch_status = 0;
  MSCCLPP_AMD_DISPATCH_ALL(dtype, op, launchBulk, views, nviews, g, nranks, nblocks, nthreads, budget, s, order, mode);
  if (g_launch_status) return g_launch_status;
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

int launchBroadcast(const mscclppAmdRankView* views, int nviews, int nranks, size_t bytes, int root, int nblocks,
                    int nthreads, uint64_t budget, hipStream_t s) {
  if (nblocks <= 0) {  // 256 KiB per workgroup, 8..128 workgroups
    const uint64_t want = (bytes + (256u << 10) - 1) / (256u << 10);
    nblocks = (int)(want < 8 ? 8 : want > 128 ? 128 : want);
  }
  if (nthreads <= 0) nthreads = 512;
  if (nblocks > kMaxChannels || nthreads > 512 || nthreads % 64 || nthreads < 64) return 4;
  if (root < 0 || root >= nranks || bytes == 0) return 4;
  const uint64_t blk = ((bytes + nblocks - 1) / nblocks + 15) & ~15ull;
  if (blk > kBlkOffsetLimit) return 5;
  auto go = [&](auto kern, auto vw) {
    if (!grid_coresident(kern, nthreads, (long)nblocks * nviews)) return 5;
    hipLaunchKernelGGL(kern, dim3(nblocks, nviews), dim3(nthreads), 0, s, vw, (uint64_t)bytes, blk, nranks, root,
                       budget);
    return hipGetLastError() == hipSuccess ? 0 : 1;
  };
  if (nviews == 1) {
    Views<1> vw;
    vw.v[0] = views[0];
    return go(broadcastKernel<1, 4>, vw);
  }
  Views<kMaxRanks> vw{};
  for (int i = 0; i < nviews; ++i) vw.v[i] = views[i];
  return go(broadcastKernel<kMaxRanks, 4>, vw);
}

template <int DT, int OP>
static void launchPipeline(const mscclppAmdRankView* views, int nviews, const PipeGeom& g, int nranks, int nthreads,
                           uint64_t budget, hipStream_t s) {
  auto go = [&](auto kern, auto vw) {
    const long blocks = (long)(g.R + g.R) * nviews;
    if (!grid_coresident(kern, nthreads, blocks)) {
      g_launch_status = 5;  // the roles wait on each other inside the launch: all must be resident
      return;
    }
    hipLaunchKernelGGL(kern, dim3(g.R + g.R, nviews), dim3(nthreads), 0, s, vw, g, nranks, budget);
  };
  if (nviews == 1) {
    Views<1> vw;
    vw.v[0] = views[0];
    go(allreduceRsAgPipelineKernel<DT, OP, 1>, vw);
  } else {
    Views<kMaxRanks> vw{};
    for (int i = 0; i < nviews; ++i) vw.v[i] = views[i];
    go(allreduceRsAgPipelineKernel<DT, OP, kMaxRanks>, vw);
  }
}

// R reduce workgroups (nblocks, even, 2..128; default 32) of nthreads (default 512) lanes; the
// scratch must hold at least one stage (2 * n * C units).
int launchAllReducePipeline(const mscclppAmdRankView* views, int nviews, int nranks, size_t bytes, int dtype, int op,
                            int nblocks, int nthreads, uint64_t budget, hipStream_t s) {
  if (nblocks <= 0) nblocks = 32;
  if (nthreads <= 0) nthreads = 512;
  if (nblocks % 2 || nblocks < 2 || nblocks > 128 || nthreads > 512 || nthreads % 64 || nthreads < 64) return 4;
  if (dtype != kF16 && dtype != kBF16 && dtype != kF32 && dtype != kI32 && dtype != kU32) return 4;
  PipeGeom g{};
  g.bytes = bytes;
  g.R = (uint32_t)nblocks;
  g.C = (uint64_t)nblocks * nthreads * 4;
  const uint64_t units = (bytes + 15) / 16;
  const uint64_t perIter = (uint64_t)nranks * g.C;
  g.nIters = (uint32_t)((units + perIter - 1) / perIter);
  const uint64_t stage = 2 * perIter * 16;
  for (int i = 0; i < nviews; ++i) {
    if (!views[i].pipeSems || !views[i].scratch) return 4;
    if (views[i].scratchBytes < stage) return 5;
  }
  // depth from the smallest view (every rank of a communicator allocates the same scratch, so the
  // stage offsets agree across ranks; in-process views may differ)
  uint64_t minScratch = views[0].scratchBytes;
  for (int i = 1; i < nviews; ++i) minScratch = views[i].scratchBytes < minScratch ? views[i].scratchBytes : minScratch;
  uint64_t D = minScratch / stage;
  g.D = (uint32_t)(D > g.nIters ? (g.nIters ? g.nIters : 1) : D);
  g_launch_status = 0;
  if (dtype == kF16)
    op == kMin ? launchPipeline<kF16, kMin>(views, nviews, g, nranks, nthreads, budget, s)
               : launchPipeline<kF16, kSum>(views, nviews, g, nranks, nthreads, budget, s);
  else if (dtype == kBF16)
    op == kMin ? launchPipeline<kBF16, kMin>(views, nviews, g, nranks, nthreads, budget, s)
               : launchPipeline<kBF16, kSum>(views, nviews, g, nranks, nthreads, budget, s);
  else if (dtype == kF32)
    op == kMin ? launchPipeline<kF32, kMin>(views, nviews, g, nranks, nthreads, budget, s)
               : launchPipeline<kF32, kSum>(views, nviews, g, nranks, nthreads, budget, s);
  else if (dtype == kI32)
    op == kMin ? launchPipeline<kI32, kMin>(views, nviews, g, nranks, nthreads, budget, s)
               : launchPipeline<kI32, kSum>(views, nviews, g, nranks, nthreads, budget, s);
  else
    op == kMin ? launchPipeline<kU32, kMin>(views, nviews, g, nranks, nthreads, budget, s)
               : launchPipeline<kU32, kSum>(views, nviews, g, nranks, nthreads, budget, s);
  if (g_launch_status) return g_launch_status;
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

int launchAllReduceBulk(int algo, const mscclppAmdRankView* views, int nviews, int nranks, size_t bytes, int dtype,
                        int op, int nblocks, int nthreads, uint64_t budget, hipStream_t s) {
  return launchCollectiveBulk(0, algo, views, nviews, nranks, bytes, dtype, op, nblocks, nthreads, budget, s);
}

}  // namespace mscclpp_amd

uint64_t* g_mscclppAmdTrace = nullptr;

extern "C" int mscclppAmdTraceSet(void* buf, size_t bytes) {
  if (buf && bytes < MSCCLPP_AMD_TRACE_BYTES) return 4;
  g_mscclppAmdTrace = (uint64_t*)buf;
  return 0;
}
