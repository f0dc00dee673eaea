// LL-packet AllReduce kernels for gfx950 over xGMI.
//
//  allreduceLL16  -- two-hop LL16 (reference: allreducePacket, src/ext/collectives/allreduce/
//                    allreduce_packet.cu:15-151).  Step 1 packs this rank's copy of slice q into
//                    rank q's scratch (one-sided put over xGMI); step 2 polls the n-1 packet
//                    streams of its own slice, sums (own first, then peers ascending), writes the
//                    result locally and broadcasts it as LL16 packets; step 3 unpacks the peers'
//                    reduced slices.  Scratch layout, flag lifecycle and sum order follow the
//                    reference exactly.
//  allreduceLL8   -- one-hop LL8 (reference: allreduceAllPairs, allreduce_allpair_packet.cu:15-69).
//                    Every rank puts its whole buffer as LL8 packets into every peer's scratch and
//                    reduces all n streams locally.
//
// Sums accumulate through Accum<DT, OP, 2> (reduce_device.hpp): the element type itself, or for
// FP8 the half / float AccumT of calVectorAccum (allreduce_packet.cu:95-108).
//
// gfx950 choices (vs. the reference's CUDA-shaped loops): one lane moves one 16-byte unit (8
// payload bytes = one LL16 packet or two LL8 packets) as a single buffer store with system-scope
// write-through (sc0 sc1), so a wave writes 1 KiB of whole lines; polls are 16-byte system-scope
// loads issued for all peers before any spin; peer
// pointers come from kernel arguments (scalar loads), not from channel handles copied to LDS; loops
// over peers are unrolled to the 8-GPU maximum with predicates so the per-peer values stay in VGPRs.
#include "common.hpp"

namespace mscclpp_amd {

struct LL16Geom {
  uint64_t bytes;   // payload bytes actually in the buffers
  uint64_t W;       // 32-bit words the algorithm covers (allreduce_packet.cu:51-54)
  uint64_t wpr;     // words per rank slice (even for allreducePacket, :62-63)
  uint64_t ppr;     // 16-byte packet units per rank slice = wpr / 2
  uint64_t roff;    // byte offset of the reduced-slice region from the input region (:74)
  uint64_t hbOdd;   // scratch byte offset of the input region when the flag is odd (:60: half)
  uint64_t hbEven;  // ... when the flag is even (:60: 0)
  uint32_t units;   // packets per slice (= ppr)
  uint32_t pad;
  uint64_t* trace;  // phase stamps (mscclppAmdTraceSet) or null
};

struct LL8Geom {
  uint64_t bytes;
  uint64_t W;       // words (= LL8 packets) per rank buffer (allreduce_allpair_packet.cu:20)
  uint32_t units;   // 2-word units = ceil(W / 2)
  uint32_t pad;
  uint64_t* trace;  // phase stamps (mscclppAmdTraceSet) or null
  uint64_t hbOdd;   // mscclpp-test allreduce2 layout only (V & 1024): scratch byte offset of the
  uint64_t hbEven;  // packets when the flag is odd / even (allreduce_test.cu:861-863)
};

// ---- packet-major units ------------------------------------------------------------------------
// One lane owns one "unit": 8 payload bytes <-> 16 packet bytes, i.e. one LL16 packet
// {P[2i], f, P[2i+1], f} or the two LL8 packets {P[2i], f}, {P[2i+1], f} -- the same 16-byte image.
// Consecutive lanes own consecutive units, so every packet store / poll of a wave is one contiguous
// 1 KiB access made of whole 64-byte lines (partial-line packet stores cost a full line each on
// gfx950: WRITE_SIZE 5*S instead of 3*S in the self-reduce microbench), and the payload side is a
// contiguous 512 B dwordx2 access.
template <int Policy>
__device__ __forceinline__ void unit_put(__amdgpu_buffer_rsrc_t pk, uint32_t pbyte, u32x2 w, uint32_t flag,
                                         bool single) {
  if (!single)
    store16<Policy>(pk, pbyte, u32x4{w.x, flag, w.y, flag});
  else
    store8<Policy>(pk, pbyte, u32x2{w.x, flag});  // lone trailing LL8 packet
}
__device__ __forceinline__ bool unit_try(__amdgpu_buffer_rsrc_t pk, uint32_t pbyte, uint32_t flag, u32x2& w,
                                         bool single) {
  if (!single) {
    u32x4 a = load16<kSystem>(pk, pbyte);
    w = u32x2{a.x, a.z};
    return a.y == flag && a.w == flag;
  }
  u32x2 a = load8<kSystem>(pk, pbyte);
  w = u32x2{a.x, 0};
  return a.y == flag;
}
// Timeout detail of one packet unit: the first of its flag words that differs from `flag`, re-read.
__device__ __forceinline__ uint32_t unit_flag_seen(__amdgpu_buffer_rsrc_t pk, uint32_t pbyte, uint32_t flag,
                                                   bool single) {
  if (single) return load8<kSystem>(pk, pbyte).y;
  const u32x4 a = load16<kSystem>(pk, pbyte);
  return a.y != flag ? a.y : a.w;
}
__device__ __forceinline__ u32x2 unit_get(__amdgpu_buffer_rsrc_t pk, uint32_t pbyte, uint32_t flag, bool single,
                                          uint64_t budget, uint32_t* err) {
  u32x2 w;
  if (unit_try(pk, pbyte, flag, w, single)) return w;
  SpinGuard g(budget);
  while (!unit_try(pk, pbyte, flag, w, single)) {
    __builtin_amdgcn_s_sleep(1);
    if (g.expired()) {
      report_packet_timeout(err, flag, pbyte, unit_flag_seen(pk, pbyte, flag, single));
      return u32x2{0, 0};
    }
  }
  return w;
}
// add_vectors<TYPE>(a, b) of python/mscclpp_benchmark/allreduce.cu:37-96 on one 8-byte payload: int
// wrapping adds, float `a + b`, __half __hadd2 -- round to nearest even and no clip (inf on overflow),
// unlike the collectives' f16x2 operator+ (gpu_data_types.hpp:389-397).
// The words are copied out of the vectors before the bit casts: this compiler (ROCm 7.2 clang)
// lowers __builtin_bit_cast of an ext_vector element such as `a.y` to a cast of element 0 -- the
// kernel then summed the first word twice (caught by tests/test_reference_kernel_gpu.py).
template <int DT>
__device__ __forceinline__ u32x2 bench_add2(u32x2 a, u32x2 b) {
  const uint32_t a0 = a.x, a1 = a.y, b0 = b.x, b1 = b.y;
  if constexpr (DT == kF16) {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const h2 s0 = __builtin_bit_cast(h2, a0) + __builtin_bit_cast(h2, b0);
    const h2 s1 = __builtin_bit_cast(h2, a1) + __builtin_bit_cast(h2, b1);
    return u32x2{__builtin_bit_cast(uint32_t, s0), __builtin_bit_cast(uint32_t, s1)};
  } else if constexpr (DT == kF32) {
    const float s0 = __builtin_bit_cast(float, a0) + __builtin_bit_cast(float, b0);
    const float s1 = __builtin_bit_cast(float, a1) + __builtin_bit_cast(float, b1);
    return u32x2{__builtin_bit_cast(uint32_t, s0), __builtin_bit_cast(uint32_t, s1)};
  } else {
    static_assert(DT == kI32 || DT == kU32, "the benchmark's allreduce2 types are int, float and __half");
    return u32x2{a0 + b0, a1 + b1};
  }
}

// First poll of unit `pbyte` in every peer's region (peer p's at p * stride of `base`): all loads
// are issued, unconditionally and in one basic block, before any value is compared, so they are in
// flight together (a compare right after each load, or a load under a branch, made the compiler wait
// for it before issuing the next: one memory round trip per peer).  A slot that is not a peer (own
// rank, p >= nranks) is loaded through a zero-length buffer resource: out of range, it returns zeros
// without touching memory.  Returns the mask of peers whose packet had not landed; w[p] holds the
// payload of the others.
__device__ __forceinline__ void poll_issue(const uint8_t* base, uint32_t stride, uint32_t pbyte, uint32_t peers,
                                           u32x4* raw) {
#pragma unroll
  for (int p = 0; p < kMaxRanks; ++p) {
    const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), 0,
                                                     ((peers >> p) & 1u) ? 0xFFFFFFFFu : 0u, 0x00020000);
    raw[p] = load16<kSystem>(r, (uint32_t)p * stride + pbyte);
  }
}
// As poll_issue, for a scratch whose source regions are indexed by peer, not by rank: source p sits
// in slot p < rank ? p : p - 1 (mscclpp-test allreduce2, allreduce_test.cu:876-880).
__device__ __forceinline__ void poll_issue_peer_slots(const uint8_t* base, uint32_t stride, uint32_t pbyte,
                                                      uint32_t peers, int rank, u32x4* raw) {
#pragma unroll
  for (int p = 0; p < kMaxRanks; ++p) {
    const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), 0,
                                                     ((peers >> p) & 1u) ? 0xFFFFFFFFu : 0u, 0x00020000);
    raw[p] = load16<kSystem>(r, (uint32_t)(p < rank ? p : p - 1) * stride + pbyte);
  }
}
__device__ __forceinline__ uint32_t poll_eval(const u32x4* raw, uint32_t flag, uint32_t peers, u32x2* w) {
  uint32_t missing = 0;
#pragma unroll
  for (int p = 0; p < kMaxRanks; ++p) {
    w[p] = u32x2{raw[p].x, raw[p].z};
    if (raw[p].y != flag || raw[p].w != flag) missing |= 1u << p;
  }
  return missing & peers;
}
__device__ __forceinline__ uint32_t poll_units(const uint8_t* base, uint32_t stride, uint32_t pbyte, uint32_t flag,
                                               uint32_t peers, u32x2* w) {
  u32x4 raw[kMaxRanks];
  poll_issue(base, stride, pbyte, peers, raw);
  return poll_eval(raw, flag, peers, w);
}
// Diagnostics build only (variant bit 32): add n, summed over the wave, to *ctr (first-poll misses).
template <int V>
__device__ __forceinline__ void count_misses(uint32_t* ctr, uint32_t n) {
  if constexpr ((V & 32) != 0) {
    for (int off = 32; off > 0; off >>= 1) n += __shfl_xor(n, off, 64);
    if ((threadIdx.x & 63) == 0 && n) __hip_atomic_fetch_add(ctr, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// A unit whose first poll missed: spin until it lands (the caller keeps the values of the units
// that were ready, so only the missing ones are read again).
__device__ __forceinline__ u32x2 unit_wait(__amdgpu_buffer_rsrc_t pk, uint32_t pbyte, uint32_t flag, bool single,
                                           uint64_t budget, uint32_t* err) {
  u32x2 w;
  SpinGuard g(budget);
  do {
    __builtin_amdgcn_s_sleep(1);
    if (unit_try(pk, pbyte, flag, w, single)) return w;
  } while (!g.expired());
  report_packet_timeout(err, flag, pbyte, unit_flag_seen(pk, pbyte, flag, single));
  return u32x2{0, 0};
}
// Wave-level readiness probe (LL16 step 3 from kSentinelUnits units per slice): one lane polls the
// last unit the wave covers in this pass (one line) until it has landed, so the wave's full poll that
// follows finds its packets there instead of re-reading lines that had not landed.  A peer stores a
// wave's 64 units with one instruction, so they land together.  On expiry it returns and the
// per-unit waits report the error.
__device__ __forceinline__ void sentinel_wait(__amdgpu_buffer_rsrc_t pk, uint32_t j, uint32_t npk, uint32_t flag,
                                              uint64_t budget) {
  const uint32_t j0 = wave_uniform(j);  // the wave's first unit (lanes hold consecutive units)
  const uint32_t js = j0 + 63 < npk ? j0 + 63 : npk - 1;
  const bool lead = (threadIdx.x & 63) == 0;
  auto probe = [&]() {
    uint32_t ok = 0;
    if (lead) {
      const u32x4 a = load16<kSystem>(pk, js * 16u);
      ok = a.y == flag && a.w == flag;
    }
    return wave_uniform(ok) != 0;
  };
  if (probe()) return;
  SpinGuard g(budget);
  do {
    __builtin_amdgcn_s_sleep(1);
    if (probe()) return;
  } while (!g.expired());
}
// 8-byte payload at byte `off` of `base`, of which `valid` bytes are inside the buffer
__device__ __forceinline__ u32x2 payload_ld(__amdgpu_buffer_rsrc_t r, const uint8_t* base, uint64_t off, uint32_t valid) {
  if (valid >= 8) return load8<kPlain>(r, (uint32_t)off);
  uint32_t w0 = 0, w1 = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if ((uint32_t)i < valid) {
      const uint32_t v = (uint32_t)base[off + i] << ((i % 4) * 8);
      if (i < 4) w0 |= v; else w1 |= v;
    }
  }
  return u32x2{w0, w1};
}
__device__ __forceinline__ void payload_st(__amdgpu_buffer_rsrc_t r, uint8_t* base, uint64_t off, u32x2 v, uint32_t valid) {
  if (valid >= 8) {
    store8<kPlain>(r, (uint32_t)off, v);
    return;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if ((uint32_t)i < valid) base[off + i] = (uint8_t)((i < 4 ? v.x : v.y) >> ((i % 4) * 8));
}

// V (0 in the product): bits that switch a part back to its round-2 form, for same-process A/B
// timing through the diagnostics build (MSCCLPP_AMD_DIAG): 4 = polls tested as issued and every peer
// re-read after a miss, 8 = a scalar flag load ahead of everything else, 16 = every slice size polls
// all peers at once, 32 = count first-poll misses into err[8] (step 2 / LL8) and err[9] (step 3),
// 64 = step 3's sentinel at every slice size, 512 = no sentinel at any size.
// Step 2 issues all of a unit's peer polls at once while a slice has at most kBatchedPollUnits units
// (LL16 buckets up to 512 KiB at 8 ranks: one memory round trip instead of one per peer, 1.0-1.5 us
// at 1-512 KiB in the A/B), and polls peer by peer beyond.
constexpr uint32_t kBatchedPollUnits = 8192;
// Step 3 waits on a one-line sentinel before a wave's first pass from this many units per slice (LL16
// buckets from 512 KiB at 8 ranks): there 15-47 % of step 3's first polls found the peer's reduced
// packet not yet landed and each re-read it (LL16 read 1.057x its algorithmic bytes at 1 MiB); with
// the sentinel none miss, and 1 MiB runs 13.8 us instead of 14.1.  Below it the sentinel's extra
// round trip costs 0.2 us (1-256 KiB) more than the re-reads it saves
// (tools/ll_variants_ab.py, profiles/r3d_ll_sentinel_ab.json).
constexpr uint32_t kSentinelUnits = 8192;
template <int DT, int OP, int NV, int V = 0>
__global__ void __launch_bounds__(512) allreduceLL16Kernel(Views<NV> views, LL16Geom g, int nranks, uint64_t budget) {
  const mscclppAmdRankView& v = views.v[NV == 1 ? 0 : blockIdx.y];
  const int rank = v.rank;
  const int nPeers = nranks - 1;
  const uint32_t T = blockDim.x, tid = threadIdx.x, G = gridDim.x, b = blockIdx.x;
  const uint8_t* in = (const uint8_t*)v.input;
  uint8_t* out = (uint8_t*)v.output;
  const auto rin = make_rsrc(in);
  const auto rout = make_rsrc(out);
  const uint64_t sliceBytes = g.wpr * 4;
  // bytes of slice q inside the buffer: the unit at byte `off` of it may carry `valid` of them
  auto sliceEnd = [&](int q) {
    const uint64_t e = (uint64_t)(q + 1) * sliceBytes;
    return e < g.bytes ? e : g.bytes;
  };
  const uint32_t npk = (uint32_t)g.ppr;          // packets (units) per slice
  const uint32_t peers = ((1u << nranks) - 1u) & ~(1u << rank);
  const uint32_t bpp = G / (uint32_t)nPeers;     // blocks per peer for steps 1 and 3
  const bool inPeerGroup = b < bpp * (uint32_t)nPeers;
  const int peerIdx = inPeerGroup ? (int)(b / bpp) : 0;
  const int remote = peerIdx < rank ? peerIdx : peerIdx + 1;
  const uint32_t lb = inPeerGroup ? b % bpp : 0;
  trace_stamp(g.trace, 0);
  // The flag is a vector load issued right before the first unit of step 1, so the two are in flight
  // together: no round trip of its own before the first put (a scalar flag load was waited for
  // before the payload load was issued).
  uint32_t flagv;
  if constexpr ((V & 8) != 0)
    flagv = v.flags[b];
  else
    flagv = __hip_atomic_load(v.flags + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t soff1 = (uint64_t)remote * sliceBytes;
  const uint64_t send1 = sliceEnd(remote);
  const uint32_t j1 = lb * T + tid;
  u32x2 w1{0, 0};
  if (inPeerGroup && j1 < npk) w1 = payload_ld(rin, in, soff1 + (uint64_t)j1 * 8, clamp_valid(send1, soff1 + (uint64_t)j1 * 8, 8));
  const uint32_t flag = wave_uniform(flagv);
  const uint64_t base = (flag & 1u) ? g.hbOdd : g.hbEven;  // numScratchBuff = 2 (allreduce_packet.cu:60)
  uint8_t* scr = (uint8_t*)v.scratch + base;

  // step 1: put my copy of slice `remote` into rank `remote`'s scratch at rank*ppr packets (:89-90)
  if (inPeerGroup) {
    const auto rdst = make_rsrc((uint8_t*)v.peerScratch[remote] + base + (uint64_t)rank * g.ppr * 16);
    for (uint32_t j = j1; j < npk; j += bpp * T) {
      const uint64_t off = soff1 + (uint64_t)j * 8;
      const u32x2 w = j == j1 ? w1 : payload_ld(rin, in, off, clamp_valid(send1, off, 8));
      unit_put<kSystem>(rdst, j * 16u, w, flag, false);
    }
  }

  trace_stamp(g.trace, 1);

  // step 2: reduce my slice from the n-1 incoming streams (own first, then peers ascending,
  // :93-106), store locally, broadcast the reduced packets (:111-122)
  {
    const auto rscr = make_rsrc(scr);
    const uint64_t soff = (uint64_t)rank * sliceBytes;
    const uint64_t send = sliceEnd(rank);
    for (uint32_t j = b * T + tid; j < npk; j += G * T) {
      const uint64_t off = soff + (uint64_t)j * 8;
      const uint32_t valid = clamp_valid(send, off, 8);
      // every peer's packet polled once and the own payload loaded, all loads in flight together
      // (issued before any value is looked at, so no wait separates them); only the peers whose
      // packet had not landed are polled again (the values of the others are kept), then the sum
      // runs in the reference order
      u32x2 w[kMaxRanks];
      uint32_t missing = 0;
      u32x2 own;
      if constexpr ((V & 4) != 0) {
        own = payload_ld(rin, in, off, valid);
        bool ready = true;
#pragma unroll
        for (int p = 0; p < kMaxRanks; ++p)
          if (p < nranks && p != rank) ready &= unit_try(rscr, (uint32_t)(p * g.ppr * 16) + j * 16u, flag, w[p], false);
        if (!ready) missing = peers;  // round 2: every peer read again
      } else if (npk > kBatchedPollUnits && (V & 16) == 0) {
        // large slices: one peer at a time, so later peers' packets have had longer to land (fewer
        // first-poll misses under load; 1 MiB: measured faster than all polls at once); a peer whose
        // packet had not landed is polled again below, the others are not re-read
        own = payload_ld(rin, in, off, valid);
#pragma unroll
        for (int p = 0; p < kMaxRanks; ++p)
          if (((peers >> p) & 1u) && !unit_try(rscr, (uint32_t)(p * g.ppr * 16) + j * 16u, flag, w[p], false))
            missing |= 1u << p;
      } else {
        u32x4 raw[kMaxRanks];
        poll_issue(scr, (uint32_t)(g.ppr * 16), j * 16u, peers, raw);
        own = payload_ld(rin, in, off, valid);
        missing = poll_eval(raw, flag, peers, w);
      }
      count_misses<V>(v.err + 8, (uint32_t)__builtin_popcount(missing));
      if (missing) {
#pragma unroll
        for (int p = 0; p < kMaxRanks; ++p)
          if ((missing >> p) & 1u) w[p] = unit_wait(rscr, (uint32_t)(p * g.ppr * 16) + j * 16u, flag, false, budget, v.err);
      }
      u32x2 acc;
      if constexpr ((V & 2048) != 0) {
        // mscclpp-test allreduce6 / the benchmark's allreduce2 (allreduce.cu:254-264): data = 0, then
        // data = val + data for the peers ascending, then data + own, each add unclipped
        acc = u32x2{0u, 0u};
#pragma unroll
        for (int p = 0; p < kMaxRanks; ++p)
          if ((peers >> p) & 1u) acc = bench_add2<DT>(w[p], acc);
        acc = bench_add2<DT>(acc, own);
      } else {
        Accum<DT, OP, 2> sum(own);  // upcastVector (:98-99)
#pragma unroll
        for (int p = 0; p < kMaxRanks; ++p)
          if ((peers >> p) & 1u) sum.add(w[p]);
        acc = sum.template get<u32x2>();  // downcastVector (:107-108)
      }
      payload_st(rout, out, off, acc, valid);
      // broadcast: a runtime loop, so one descriptor is live at a time (SGPR budget)
#pragma unroll 1
      for (int q = 0; q < nranks; ++q) {
        if (q == rank) continue;
        const auto rq = make_rsrc((uint8_t*)v.peerScratch[q] + base + g.roff + (uint64_t)rank * g.ppr * 16);
        unit_put<kSystem>(rq, j * 16u, acc, flag, false);
      }
    }
  }

  trace_stamp(g.trace, 2);

  // step 3: unpack the reduced slice of peer `remote` (:125-132)
  if (inPeerGroup) {
    const auto rres = make_rsrc(scr + g.roff + (uint64_t)remote * g.ppr * 16);
    const uint64_t soff = (uint64_t)remote * sliceBytes;
    const uint64_t send = sliceEnd(remote);
    // one unit per lane and pass, polled and then waited for: issuing a lane's later passes' polls
    // together with its first (all reading lines that had not landed yet) measured slower at every
    // size in the same-process A/B (tools/ll_variants_ab.py, profiles/r3_ll_variants_ab.json)
    const bool sentinel = (V & 512) == 0 && ((V & 64) != 0 || npk >= kSentinelUnits);
    for (uint32_t j = lb * T + tid; j < npk; j += bpp * T) {
      const uint64_t off = soff + (uint64_t)j * 8;
      if (sentinel && j < (lb + 1) * T) sentinel_wait(rres, j, npk, flag, budget);  // the wave's first pass
      u32x2 w;
      const bool landed = unit_try(rres, j * 16u, flag, w, false);
      count_misses<V>(v.err + 9, landed ? 0u : 1u);
      if (!landed) w = unit_wait(rres, j * 16u, flag, false, budget, v.err);
      payload_st(rout, out, off, w, clamp_valid(send, off, 8));
    }
  }
  trace_stamp(g.trace, 3);
  bump_flags(v.flags, flag);
}

// V: as allreduceLL16Kernel's (bits 4 and 8); 1024 = mscclpp-test allreduce2 on one node
// (allreduce_test.cu:841-943): the same one hop with the harness's scratch -- source regions indexed
// by peer (p < rank ? p : p - 1), odd flags at 0 and even ones after the n - 1 regions.  Its
// LLPacket {x, flag, y, flag} is the 16-byte unit image below; int32, even nelems (the host checks).
template <int DT, int OP, int NV, int V = 0>
__global__ void __launch_bounds__(512) allreduceLL8Kernel(Views<NV> views, LL8Geom g, int nranks, uint64_t budget) {
  const mscclppAmdRankView& v = views.v[NV == 1 ? 0 : blockIdx.y];
  const int rank = v.rank;
  const uint32_t T = blockDim.x, G = gridDim.x;
  const uint32_t gtid = blockIdx.x * T + threadIdx.x;
  const uint8_t* in = (const uint8_t*)v.input;
  uint8_t* out = (uint8_t*)v.output;
  const auto rin = make_rsrc(in);
  const auto rout = make_rsrc(out);
  const uint64_t region = g.W * 8;  // LL8 bytes one source rank occupies in a peer's scratch half
  const uint32_t peers = ((1u << nranks) - 1u) & ~(1u << rank);
  trace_stamp(g.trace, 0);
  // The flag is a vector load issued right before this lane's first payload load, so the two are in
  // flight together (one memory round trip before the first put, where a scalar flag load was waited
  // for before the payload load was issued); the payload is also the own term of that unit's sum.
  uint32_t flagv;
  if constexpr ((V & 8) != 0)
    flagv = v.flags[blockIdx.x];
  else
    flagv = __hip_atomic_load(v.flags + blockIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  u32x2 w0{0, 0};
  if (gtid < g.units) {
    const bool single = 2ull * gtid + 1 >= g.W;
    w0 = payload_ld(rin, in, (uint64_t)gtid * 8, clamp_valid(g.bytes, (uint64_t)gtid * 8, single ? 4 : 8));
  }
  const uint32_t flag = wave_uniform(flagv);
  constexpr bool kPeerSlots = (V & 1024) != 0;
  const uint64_t base = kPeerSlots ? ((flag & 1u) ? g.hbOdd : g.hbEven) : ((flag & 1u) ? v.scratchBytes / 2 : 0);
  // byte offset of source p's region in a scratch half
  auto slotOff = [&](int p) -> uint32_t { return (uint32_t)((kPeerSlots && p > rank ? p - 1 : p) * region); };

  // put my whole buffer into every peer's scratch at rank*W packets (allreduce_allpair_packet.cu:39-42)
  for (uint32_t j = gtid; j < g.units; j += G * T) {
    const bool single = 2ull * j + 1 >= g.W;
    const uint64_t off = (uint64_t)j * 8;
    const u32x2 w = j == gtid ? w0 : payload_ld(rin, in, off, clamp_valid(g.bytes, off, single ? 4 : 8));
#pragma unroll 1
    for (int q = 0; q < nranks; ++q) {
      if (q == rank) continue;
      const uint64_t mySlot = kPeerSlots && rank > q ? rank - 1 : rank;  // my region in q's scratch
      const auto rq = make_rsrc((uint8_t*)v.peerScratch[q] + base + mySlot * region);
      unit_put<kSystem>(rq, j * 16u, w, flag, single);
    }
  }
  trace_stamp(g.trace, 1);
  // reduce: own first, then peers ascending (:49-61).  The same lane handled unit j above, so an
  // in-place call reads its input before overwriting it.
  const auto rscr = make_rsrc((uint8_t*)v.scratch + base);
  for (uint32_t j = gtid; j < g.units; j += G * T) {
    const bool single = 2ull * j + 1 >= g.W;
    const uint64_t off = (uint64_t)j * 8;
    const uint32_t valid = clamp_valid(g.bytes, off, single ? 4 : 8);
    Accum<DT, OP, 2> sum(j == gtid ? w0 : payload_ld(rin, in, off, valid));  // upcastVector (:54)
    u32x2 w[kMaxRanks];
    // peers whose packet had not landed at the first poll: only those are re-polled.  The waves
    // without the lone trailing LL8 packet (all but at most one) poll 16-byte units with every load
    // issued before any value is looked at; the one that has it takes the per-lane path.
    const uint32_t jw = wave_uniform(j);  // the wave's first unit (lanes hold consecutive units)
    const bool waveSingle = (g.W & 1) && 2ull * (jw + 63) + 1 >= g.W;
    uint32_t missing = 0;
    if constexpr ((V & 4) != 0) {
      bool ready = true;
#pragma unroll
      for (int p = 0; p < kMaxRanks; ++p)
        if (p < nranks && p != rank) ready &= unit_try(rscr, slotOff(p) + j * 16u, flag, w[p], single);
      if (!ready) missing = peers;  // round 2: every peer read again
    } else if (kPeerSlots) {
      u32x4 raw[kMaxRanks];
      poll_issue_peer_slots((const uint8_t*)v.scratch + base, (uint32_t)region, j * 16u, peers, rank, raw);
      missing = poll_eval(raw, flag, peers, w);
    } else if (!waveSingle) {
      missing = poll_units((const uint8_t*)v.scratch + base, (uint32_t)region, j * 16u, flag, peers, w);
    } else {
#pragma unroll
      for (int p = 0; p < kMaxRanks; ++p)
        if (((peers >> p) & 1u) && !unit_try(rscr, slotOff(p) + j * 16u, flag, w[p], single))
          missing |= 1u << p;
    }
    count_misses<V>(v.err + 8, (uint32_t)__builtin_popcount(missing));
    if (missing) {
#pragma unroll
      for (int p = 0; p < kMaxRanks; ++p)
        if ((missing >> p) & 1u) w[p] = unit_wait(rscr, slotOff(p) + j * 16u, flag, single, budget, v.err);
    }
#pragma unroll
    for (int p = 0; p < kMaxRanks; ++p)
      if ((peers >> p) & 1u) sum.add(w[p]);
    payload_st(rout, out, off, sum.template get<u32x2>(), valid);  // downcastVector (:61)
  }
  trace_stamp(g.trace, 2);
  bump_flags(v.flags, flag);
}

// ---- host-side geometry + launch -------------------------------------------------------------------
// 32-bit words the LL kernels cover: (count*sizeof(T)+sizeof(T))/sizeof(int) for 1- and 2-byte T
// (allreduce_packet.cu:51-52, allreduce_allpair_packet.cu:20).  Deviation: for 1-byte T with
// count % 4 in {1, 2} that stops short of the buffer (its last bytes would never be reduced), so
// the words are rounded up there; every other size keeps the reference's count.
static inline uint64_t llWords(size_t bytes, int dtype) {
  const int es = elem_bytes(dtype);
  if (es == 4) return bytes / 4;
  uint64_t W = (bytes + es) / 4;
  if (W * 4 < bytes) W = (bytes + 3) / 4;
  return W;
}

static LL16Geom ll16Geometry(int nranks, size_t bytes, int dtype) {
  LL16Geom g{};
  g.trace = g_mscclppAmdTrace;
  g.bytes = bytes;
  g.W = llWords(bytes, dtype);
  g.wpr = g.W / (uint64_t)nranks;
  if (g.wpr % 2) g.wpr += 1;
  // Deviation from allreduce_packet.cu:62-63: when W % n != 0 and W / n is even the reference's
  // slices stop short of W and its last words are never reduced.  Widen the slice by one packet
  // pair in exactly that case; every size the reference handles correctly keeps its geometry.
  if (g.wpr * (uint64_t)nranks < g.W) g.wpr += 2;
  g.ppr = g.wpr / 2;
  g.roff = 2 * (g.W / 2) * 16;  // scratchResultOffset (:74)
  // Deviation: when the slices were rounded up (odd W / n, or the tail fix above) the last
  // source's input packets would overlap the first reduced slice and a fast rank's broadcast could
  // overwrite packets not yet consumed.  Start the result region after the input region then.
  if ((uint64_t)nranks * g.ppr * 16 > g.roff) g.roff = (uint64_t)nranks * g.ppr * 16;
  g.units = (uint32_t)g.ppr;
  return g;
}

static LL8Geom ll8Geometry(size_t bytes, int dtype) {
  LL8Geom g{};
  g.trace = g_mscclppAmdTrace;
  g.bytes = bytes;
  g.W = llWords(bytes, dtype);
  g.units = (uint32_t)((g.W + 1) / 2);
  return g;
}

// mscclpp-test kernels 6 / 7 (test/mscclpp-test/allreduce_test.cu:972-1093): the same two-hop
// algorithm on int32 with the harness's own scratch layout -- no slice rounding
// (nelemsPerRank = nelems / worldSize), input region at packet (flag & 1 ? 0 : nPkts) and result
// region at (flag & 1 ? 2 : 3) * nPkts (:987-991, :1048-1051).  k7 moves LL8 packets; two
// consecutive LL8 packets are byte-identical to one LL16 packet of the same payload, and k7's
// offsets in 8-byte packets equal k6's in 16-byte packets, so with an even nelemsPerRank both
// scratch images are exactly those of this kernel.  Restriction (checked by the host): bytes is a
// multiple of 8 * nranks.
static bool testLLGeometry(int nranks, size_t bytes, LL16Geom* out) {
  if (bytes == 0 || bytes % (8 * (size_t)nranks)) return false;
  LL16Geom g{};
  g.trace = g_mscclppAmdTrace;
  g.bytes = bytes;
  g.W = bytes / 4;
  g.wpr = g.W / nranks;
  g.ppr = g.wpr / 2;
  const uint64_t nPkts = g.W / 2;
  g.roff = 2 * nPkts * 16;
  g.hbOdd = 0;
  g.hbEven = nPkts * 16;
  g.units = (uint32_t)g.ppr;
  *out = g;
  return true;
}

// mscclpp-test allreduce2 on one node (allreduce_test.cu:841-943): int32 pairs, nelems even -> bytes
// a multiple of 8; each half of the scratch holds n - 1 regions of nPkts = nelems / 2 LLPackets.
static bool testK2Geometry(int nranks, size_t bytes, LL8Geom* out) {
  if (bytes == 0 || bytes % 8) return false;
  LL8Geom g{};
  g.trace = g_mscclppAmdTrace;
  g.bytes = bytes;
  g.W = bytes / 4;
  g.units = (uint32_t)(g.W / 2);
  g.hbOdd = 0;
  g.hbEven = (uint64_t)g.units * 16 * (uint64_t)(nranks - 1);  // scratchBaseIndex = nPkts * nPeers
  *out = g;
  return true;
}

// The LL kernels address a buffer, and all source regions of a scratch half, from one buffer
// resource each (32-bit offsets: the whole packet exchange of a bucket stays in one descriptor, no
// per-unit rebasing on the latency path).  So an LL bucket is bounded: its bytes, and the n regions
// of a scratch half, must lie within 4 GiB of their base -- LL16 to just under 2 GiB per rank,
// LL8 to 2 GiB / n; beyond, the call is refused (ncclInvalidUsage) rather than wrapped.  The
// reference runs these protocols below 1 MiB (algorithm_selector.cc:107-117); larger buckets take the
// bulk paths, which rebase per workgroup and per pass.
constexpr uint64_t kLLOffsetLimit = 0xFFFFFFFFull - 64;
static bool ll16Fits(int nranks, const LL16Geom& g) {
  return g.bytes <= kLLOffsetLimit && (uint64_t)nranks * g.ppr * 16 <= kLLOffsetLimit;
}
static bool ll8Fits(int nranks, const LL8Geom& g) {
  return g.bytes <= kLLOffsetLimit && (uint64_t)nranks * g.W * 8 + 16 <= kLLOffsetLimit;
}

size_t testK2ScratchRequired(int nranks, size_t bytes) {
  LL8Geom g;
  if (!testK2Geometry(nranks, bytes, &g) || !ll8Fits(nranks, g)) return 0;
  return 2 * g.hbEven;  // nPacket * max(nRanksPerNode - 1, 1) * 2 LLPackets (:1277-1283)
}

size_t testLLScratchRequired(int nranks, size_t bytes) {
  LL16Geom g;
  if (!testLLGeometry(nranks, bytes, &g) || !ll16Fits(nranks, g)) return 0;
  return 4 * (g.W / 2) * 16;  // nPacket * 2 (data, result) * 2 (double buffering), :1282-1286
}

size_t ll16ScratchRequired(int nranks, size_t bytes, int dtype) {
  LL16Geom g = ll16Geometry(nranks, bytes, dtype);
  if (g.W == 0 || !ll16Fits(nranks, g)) return 0;
  uint64_t half = g.roff + (uint64_t)nranks * g.ppr * 16;
  const uint64_t inRegion = (uint64_t)nranks * g.ppr * 16;
  if (inRegion > half) half = inRegion;
  half = (half + 255) & ~255ull;
  return 2 * half;
}

size_t ll8ScratchRequired(int nranks, size_t bytes, int dtype) {
  LL8Geom g = ll8Geometry(bytes, dtype);
  if (g.W == 0 || !ll8Fits(nranks, g)) return 0;
  uint64_t half = ((uint64_t)nranks * g.W * 8 + 255) & ~255ull;
  return 2 * half;
}

static thread_local int g_ll_launch_status = 0;

template <int DT, int OP, int NV, int V = 0>
static void launchLL16T(const Views<NV>& vw, int nviews, const LL16Geom& g, int nranks, int nblocks, int nthreads, uint64_t budget,
                        hipStream_t s) {
  if (!grid_coresident(allreduceLL16Kernel<DT, OP, NV, V>, nthreads, (long)nblocks * nviews)) {
    g_ll_launch_status = 5;  // ncclInvalidUsage: the grid cannot be resident at once: its packet waits would deadlock
    return;
  }
  hipLaunchKernelGGL((allreduceLL16Kernel<DT, OP, NV, V>), dim3(nblocks, nviews), dim3(nthreads), 0, s, vw, g, nranks, budget);
}
template <int DT, int OP, int NV, int V = 0>
static void launchLL8T(const Views<NV>& vw, int nviews, const LL8Geom& g, int nranks, int nblocks, int nthreads, uint64_t budget,
                       hipStream_t s) {
  if (!grid_coresident(allreduceLL8Kernel<DT, OP, NV, V>, nthreads, (long)nblocks * nviews)) {
    g_ll_launch_status = 5;  // ncclInvalidUsage: the grid cannot be resident at once: its packet waits would deadlock
    return;
  }
  hipLaunchKernelGGL((allreduceLL8Kernel<DT, OP, NV, V>), dim3(nblocks, nviews), dim3(nthreads), 0, s, vw, g, nranks, budget);
}

template <int DT, int OP>
static void launchLL16(const mscclppAmdRankView* views, int nviews, const LL16Geom& g, int nranks, int nblocks,
                       int nthreads, uint64_t budget, hipStream_t s) {
  if (nviews == 1) {
    Views<1> vw;
    vw.v[0] = views[0];
    launchLL16T<DT, OP, 1>(vw, nviews, g, nranks, nblocks, nthreads, budget, s);
  } else {
    Views<kMaxRanks> vw{};
    for (int i = 0; i < nviews; ++i) vw.v[i] = views[i];
    launchLL16T<DT, OP, kMaxRanks>(vw, nviews, g, nranks, nblocks, nthreads, budget, s);
  }
}
template <int DT, int OP, int V = 0>
static void launchLL8(const mscclppAmdRankView* views, int nviews, const LL8Geom& g, int nranks, int nblocks,
                      int nthreads, uint64_t budget, hipStream_t s) {
  if (nviews == 1) {
    Views<1> vw;
    vw.v[0] = views[0];
    launchLL8T<DT, OP, 1, V>(vw, nviews, g, nranks, nblocks, nthreads, budget, s);
  } else {
    Views<kMaxRanks> vw{};
    for (int i = 0; i < nviews; ++i) vw.v[i] = views[i];
    launchLL8T<DT, OP, kMaxRanks, V>(vw, nviews, g, nranks, nblocks, nthreads, budget, s);
  }
}
// mscclpp-test allreduce6 / allreduce7 and the benchmark's allreduce2: the LL16 kernel with the harness
// geometry and the benchmark's sum order (V 2048).  int32 for the harness kernels; fp16 and fp32 as the
// benchmark builds allreduce2 with TYPE=__half / float.
template <int DT, int OP>
static void launchTestK6(const mscclppAmdRankView* views, int nviews, const LL16Geom& g, int nranks, int nblocks,
                         int nthreads, uint64_t budget, hipStream_t s) {
  if constexpr ((DT == kI32 || DT == kU32 || DT == kF16 || DT == kF32) && OP == kSum) {
    if (nviews == 1) {
      Views<1> vw;
      vw.v[0] = views[0];
      launchLL16T<DT, OP, 1, 2048>(vw, nviews, g, nranks, nblocks, nthreads, budget, s);
    } else {
      Views<kMaxRanks> vw{};
      for (int i = 0; i < nviews; ++i) vw.v[i] = views[i];
      launchLL16T<DT, OP, kMaxRanks, 2048>(vw, nviews, g, nranks, nblocks, nthreads, budget, s);
    }
  } else {
    launchLL16<DT, OP>(views, nviews, g, nranks, nblocks, nthreads, budget, s);  // int32 MIN: order-free
  }
}
template <int DT, int OP>
static void launchTestK2(const mscclppAmdRankView* views, int nviews, const LL8Geom& g, int nranks, int nblocks,
                         int nthreads, uint64_t budget, hipStream_t s) {
  launchLL8<DT, OP, 1024>(views, nviews, g, nranks, nblocks, nthreads, budget, s);
}

// Default grids.  LL16: a multiple of the peer count (allreduce_packet.cu:164; its defaults, :180-212,
// are (n-1)*4 blocks below 32 KiB and (n-1)*8 above).  Restated for this kernel from the fabric-free
// sweep (tools/inprocess_ll_probe.py, profiles/r2g_inprocess_ll_probe.json, 8 ranks): steps 1 and 3
// move a peer's slice with G/(n-1) blocks, and every extra pass over it adds a poll round trip, so
// the blocks per peer cover the slice in one pass, from 4 up to max(16, 48 / (n-1)) per peer and at
// most 56 in all; 512 lanes below 32 KiB and from 256 KiB, 256 between.  (Round 3, the same sweep at 2,
// 3 and 4 ranks, profiles/r3f_inprocess_ll_probe_n{2,3,4}.json: with few peers the round-2 cap of 16
// blocks per peer left a large slice to several passes -- 2 ranks at 1 MiB 19.3 us on 16 blocks, 9.5 us
// on 56; 3 ranks 14.0 us on 32, 10.7 on 48; 4 ranks already at its best on 48.)
static void ll16Defaults(int nranks, size_t bytes, int& nblocks, int& nthreads) {
  const int nPeers = nranks - 1;
  const LL16Geom g = ll16Geometry(nranks, bytes, kF16);
  if (nthreads <= 0) nthreads = (bytes < (32u << 10) || bytes >= (256u << 10)) ? 512 : 256;
  if (nblocks <= 0) {
    const uint64_t bppMax = 48 / nPeers > 16 ? 48 / nPeers : 16;
    uint64_t bpp = (g.units + nthreads - 1) / nthreads;  // blocks per peer for one pass
    if (bpp < 4) bpp = 4;
    if (bpp > bppMax) bpp = bppMax;
    while (bpp > 1 && bpp * nPeers > 56) --bpp;
    nblocks = (int)(bpp * nPeers);
  }
  nblocks = nblocks / nPeers * nPeers;
  if (nblocks < nPeers) nblocks = nPeers;
}

// LL8: one lane per 16-byte unit, up to 128 workgroups; 256 lanes up to 128 KiB, 512 above (round 3:
// at 2 ranks, where the selector keeps the one-hop form up to 1 MiB, the round-2 cap of 64 x 256 lanes
// left 512 KiB - 1 MiB to 2-4 passes: 8.7 / 15.1 us against 4.4 / 6.2 us on 128 x 512,
// profiles/r3n_inprocess_ll8_probe_n2_shapes.json).
static void ll8Defaults(int nranks, size_t bytes, int& nblocks, int& nthreads) {
  const LL8Geom g = ll8Geometry(bytes, kF16);
  if (nthreads <= 0) nthreads = g.units <= 16384 ? 256 : 512;
  if (nblocks <= 0) {
    uint64_t want = (g.units + nthreads - 1) / nthreads;
    if (want < 1) want = 1;
    if (want > 128) want = 128;
    nblocks = (int)want;
  }
  (void)nranks;
}

int launchAllReduceLL(int algo, const mscclppAmdRankView* views, int nviews, int nranks, size_t bytes, int dtype,
                      int op, int nblocks, int nthreads, uint64_t budget, hipStream_t s) {
  g_ll_launch_status = 0;
  if (algo == MSCCLPP_AMD_ALGO_PACKET) {
    // an explicit grid narrower than the peer count is an invalid argument (allreduce_packet.cu:238-241)
    if (nblocks > 0 && nblocks < nranks - 1) return 4;
    ll16Defaults(nranks, bytes, nblocks, nthreads);
    if (nblocks > kFlagSlots || nthreads > 512 || nthreads % 64) return 4;
    LL16Geom g = ll16Geometry(nranks, bytes, dtype);
    if (g.W == 0) return 4;
    if (!ll16Fits(nranks, g)) return 5;
    for (int i = 0; i < nviews; ++i)
      if (views[i].scratchBytes != views[0].scratchBytes || views[i].scratchBytes < ll16ScratchRequired(nranks, bytes, dtype))
        return 5;
    g.hbOdd = views[0].scratchBytes / 2;  // (flag % numScratchBuff) ? scratchBufferSize / 2 : 0 (:60)
    g.hbEven = 0;
    MSCCLPP_AMD_DISPATCH_ALL(dtype, op,launchLL16, views, nviews, g, nranks, nblocks, nthreads, budget, s);
  } else if (algo == MSCCLPP_AMD_ALGO_TEST_K2) {
    // harness default (allreduce_test.cu:1142-1145): (nRanksPerNode - 1) blocks of 1024 threads ->
    // twice as many 512-lane workgroups here
    if (nthreads <= 0) nthreads = 512;
    if (nblocks <= 0) nblocks = 2 * (nranks - 1);
    if (nblocks > kFlagSlots || nthreads > 512 || nthreads % 64) return 4;
    if (dtype != kI32 && dtype != kU32) return 4;  // an int32 AllReduce
    LL8Geom g;
    if (!testK2Geometry(nranks, bytes, &g) || !ll8Fits(nranks, g)) return 5;
    for (int i = 0; i < nviews; ++i)
      if (views[i].scratchBytes < testK2ScratchRequired(nranks, bytes)) return 5;
    MSCCLPP_AMD_DISPATCH(dtype, op, launchTestK2, views, nviews, g, nranks, nblocks, nthreads, budget, s);
  } else if (algo == MSCCLPP_AMD_ALGO_TEST_K6 || algo == MSCCLPP_AMD_ALGO_TEST_K7) {
    // harness defaults (allreduce_test.cu:1134-1141): k6 21 x 512, k7 28 x 1024 -> 512-lane waves here
    if (nthreads <= 0) nthreads = 512;
    if (nblocks <= 0) nblocks = algo == MSCCLPP_AMD_ALGO_TEST_K6 ? 21 : 28;
    nblocks = nblocks / (nranks - 1) * (nranks - 1);
    if (nblocks < nranks - 1) nblocks = nranks - 1;
    if (nblocks > kFlagSlots || nthreads > 512 || nthreads % 64) return 4;
    // the mscclpp-test kernels are int32 AllReduces; k6 also runs fp16 / fp32 SUM as the benchmark's
    // allreduce2 (python/mscclpp_benchmark/allreduce.cu:223-289, TYPE=__half / float) does
    const bool benchTyped = algo == MSCCLPP_AMD_ALGO_TEST_K6 && (dtype == kF16 || dtype == kF32) && op == kSum;
    if (dtype != kI32 && dtype != kU32 && !benchTyped) return 4;
    LL16Geom g;
    if (!testLLGeometry(nranks, bytes, &g) || !ll16Fits(nranks, g)) return 5;
    for (int i = 0; i < nviews; ++i)
      if (views[i].scratchBytes < testLLScratchRequired(nranks, bytes)) return 5;
    if (dtype == kF16)
      launchTestK6<kF16, kSum>(views, nviews, g, nranks, nblocks, nthreads, budget, s);
    else if (dtype == kF32)
      launchTestK6<kF32, kSum>(views, nviews, g, nranks, nblocks, nthreads, budget, s);
    else
      MSCCLPP_AMD_DISPATCH(dtype, op, launchTestK6, views, nviews, g, nranks, nblocks, nthreads, budget, s);
  } else {
    ll8Defaults(nranks, bytes, nblocks, nthreads);
    if (nblocks > kFlagSlots || nthreads > 512 || nthreads % 64) return 4;
    const LL8Geom g = ll8Geometry(bytes, dtype);
    if (g.W == 0) return 4;
    if (!ll8Fits(nranks, g)) return 5;
    for (int i = 0; i < nviews; ++i)
      if (views[i].scratchBytes < ll8ScratchRequired(nranks, bytes, dtype)) return 5;
    MSCCLPP_AMD_DISPATCH_ALL(dtype, op,launchLL8, views, nviews, g, nranks, nblocks, nthreads, budget, s);
  }
  if (g_ll_launch_status) return g_ll_launch_status;
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

}  // namespace mscclpp_amd

#ifdef MSCCLPP_AMD_DIAG
// Same-process A/B timing of the LL kernels' variants (fp16 SUM; the diagnostics library
// tests/bin/libll_diag.so only): algo MSCCLPP_AMD_ALGO_PACKET / _ALLPAIR, variant bits as V above
// (0, 4, 8, 12), views of nviews in-process ranks, default launch shape for nblocks = nthreads = 0.
uint64_t* g_mscclppAmdTrace = nullptr;
using namespace mscclpp_amd;
extern "C" int mscclppAmdDiagAllReduceLL(int algo, const mscclppAmdRankView* views, int nviews, int nranks,
                                         size_t bytes, int nblocks, int nthreads, int variant, uint64_t budget,
                                         void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (nviews != nranks || nranks < 2 || nranks > kMaxRanks) return 4;
  Views<kMaxRanks> vw{};
  for (int i = 0; i < nviews; ++i) vw.v[i] = views[i];
  g_ll_launch_status = 0;
  if (algo == MSCCLPP_AMD_ALGO_PACKET) {
    // an explicit grid narrower than the peer count is an invalid argument (allreduce_packet.cu:238-241)
    if (nblocks > 0 && nblocks < nranks - 1) return 4;
    ll16Defaults(nranks, bytes, nblocks, nthreads);
    LL16Geom g = ll16Geometry(nranks, bytes, kF16);
    if (views[0].scratchBytes < ll16ScratchRequired(nranks, bytes, kF16)) return 5;
    g.hbOdd = views[0].scratchBytes / 2;
    g.hbEven = 0;
#define LV(VV) if (variant == VV) launchLL16T<kF16, kSum, kMaxRanks, VV>(vw, nviews, g, nranks, nblocks, nthreads, budget, s);
    LV(0) LV(4) LV(8) LV(12) LV(16) LV(32) LV(48) LV(64) LV(96) LV(512) LV(544)
#undef LV
  } else if (algo == MSCCLPP_AMD_ALGO_ALLPAIR) {
    ll8Defaults(nranks, bytes, nblocks, nthreads);
    const LL8Geom g = ll8Geometry(bytes, kF16);
    if (views[0].scratchBytes < ll8ScratchRequired(nranks, bytes, kF16)) return 5;
#define LV(VV) if (variant == VV) launchLL8T<kF16, kSum, kMaxRanks, VV>(vw, nviews, g, nranks, nblocks, nthreads, budget, s);
    LV(0) LV(4) LV(8) LV(12) LV(32)
#undef LV
  } else {
    return 4;
  }
  if (g_ll_launch_status) return g_ll_launch_status;
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
#endif
