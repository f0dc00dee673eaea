// 1-GPU LL16 self-reduce microbench (BASELINE.json configs[1]).
//
//   P = LL16(Y, flag)                 pack   (copyToPackets<LL16>, copy_device.hpp:160-171)
//   O = X (op) unpack(P, flag)        reduce (LL16Packet::read + calVectorAccum, allreduce_packet.cu:93-108)
//
// One launch, two roles per wave.  Wave w of workgroup b packs its 1 KiB chunks of tile t = i*G + b
// in round i and consumes the chunks its partner packed -- purely through the LL flags in the
// packet buffer in memory, as a peer GPU's packets arrive in the AllReduce.  The partner is the
// neighbouring wave w ^ 1 of the same workgroup (round 4, PMASK 0).  Rounds 1-3 paired workgroup b
// with b ^ 1 on another XCD (blocks are dealt round-robin over the 8 XCDs); the packets crossed no
// more memory that way, but every consumer then also waited for a workgroup the dispatcher had
// started up to ~0.6 us later: 0.6-2 us of a 3-8 us one-round bucket and 2.5 us at 8 MiB
// (profiles/r4a_small_bucket_probe*.json, r4a_multi_round_probe.json; the b ^ 1 and b ^ 8 forms
// stay in the diagnostics library).  With SKEW the chunk consumed in round i is the one the partner
// packed in round i - SKEW: it has had a round to land, so the first poll finds its flags and no
// uncached 1 KiB packet line is re-read (profiles/r1f_*).  Every spin is time-bounded; a partner
// lives in the same workgroup, so no residency requirement is left.
//
// Algorithmic HBM bytes per launch: 7*S (Y read S, P written 2S, P read 2S, X read S, O written S).
#include "common.hpp"

namespace mscclpp_amd {

// LDS-staged packets: the payload side moves 16 bytes per lane (one dwordx4 per wave instruction,
// 1 KiB per wave) and the packet side stays packet-major (lane j owns packet j).  A wave turns its
// 1 KiB of payload into 128 packets through 1 KiB of its own LDS: each lane writes its 16 bytes, then
// reads back the 8 bytes of packet j and of packet 64 + j; the consumer runs the same swizzle in
// reverse before the 16-byte-per-lane sum and output store.  LDS traffic per wave-tile is three
// ds ops per side; the crossing stays inside one wave, so no barrier is needed (one wave's LDS
// operations complete in order).  The pack side and the consume side use separate LDS tiles, so
// with SKEW the consume of one tile and the pack of another never share a buffer.
//
// COUNT: diagnostic build that adds the number of packets whose first poll missed to pollMiss[0]
// (one atomic per wave and round), to measure the re-poll traffic the skew removes.
//
// W waves per workgroup, U KiB of payload per wave and round.  Large buckets: W = 4, U = 2 on 1024
// workgroups.  Small buckets are latency-bound (a few dependent memory round trips): 1 KiB per wave
// and one round, so the chain is X / Y loads -> packet stores -> partner's polls -> output stores,
// with no drain round (SKEW only pays from 3 rounds on).
// The flag is read by a vector load issued with the first payload loads, so its latency overlaps
// theirs instead of preceding them (a scalar flag load made the kernel wait for it before issuing
// anything else).
// LP: cache policy of the X / Y payload loads and the output stores (nt for streaming buckets; the
// one-round small form reads with the default policy, so a bucket written or read just before --
// an AllReduce's input straight from its producer kernel -- is served from the caches).
//
// PMASK: workgroup b's partner is b ^ PMASK (1: the neighbour, on another XCD; 8: the same XCD).
// TR: diagnostic build that stamps lane 0 of wave 0's wall clock into trace[b * 8 + event] (pollMiss
// is then a uint64_t trace buffer): 0 start, 1 payload loads landed, 2 packet stores acknowledged,
// 3 partner's packets ready, 4 output stores acknowledged, 5 flags bumped.  Each stamp waits for the
// wave's outstanding memory operations first, so the phases are serialised (diagnosis only).
template <int DT, int OP, int W, int U, int SKEW, bool COUNT, int LP = kNonTemporal, int PMASK = 1, bool TR = false>
__global__ void __launch_bounds__(64 * W) selfReduceLL16LdsKernel(const uint8_t* __restrict__ x,
                                                                  const uint8_t* __restrict__ y, uint8_t* pkts,
                                                                  uint8_t* __restrict__ out, uint64_t bytes,
                                                                  uint32_t* flags, uint64_t budget, uint32_t* err,
                                                                  uint32_t* pollMiss) {
  auto stamp = [&](int ev) {
    if constexpr (TR) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      if (threadIdx.x == 0) ((uint64_t*)pollMiss)[blockIdx.x * 8 + ev] = wall_ticks();
    }
  };
  stamp(0);
  constexpr uint32_t kWaves = W;
  constexpr uint64_t kTileBytes = (uint64_t)kWaves * U * 1024;  // payload bytes per workgroup and round
  __shared__ __attribute__((aligned(16))) uint8_t ldsP[kWaves][U][1024];
  __shared__ __attribute__((aligned(16))) uint8_t ldsC[kWaves][U][1024];
  const uint32_t G = gridDim.x, b = blockIdx.x;
  const uint32_t wave = wave_uniform(threadIdx.x / 64), lane = threadIdx.x % 64;  // wave-uniform: scalar rsrc
  const uint64_t ntiles = (bytes + kTileBytes - 1) / kTileBytes;
  const uint64_t rounds = (ntiles + G - 1) / G;
  // PMASK 0: the partner is this workgroup itself and wave w consumes the chunks wave w ^ 1 packed
  // (same CU); otherwise workgroup b ^ PMASK, wave for wave
  const uint32_t partner = b ^ (uint32_t)PMASK;
  const uint32_t cwave = PMASK == 0 ? (wave ^ 1u) : wave;
  // payload byte offset of (tile, sub-tile k) for this wave: 1 KiB chunks dealt k-major over waves
  auto chunk = [&](uint64_t t, int k) { return t * kTileBytes + (uint64_t)(k * kWaves + wave) * 1024; };
  auto cchunk = [&](uint64_t t, int k) { return t * kTileBytes + (uint64_t)(k * kWaves + cwave) * 1024; };
  u32x4 yw[U];
  auto load_y = [&](uint64_t t) {
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint64_t c = chunk(t, k);
      if (c + lane * 16 < bytes) yw[k] = load16<LP>(make_rsrc(y + c), lane * 16);
    }
  };
  u32x4 a[U];
  auto load_x = [&](uint64_t tp) {
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint64_t c = cchunk(tp, k);
      if (c + lane * 16 < bytes) a[k] = load16<LP>(make_rsrc(x + c), lane * 16);
    }
  };
  const uint32_t flagv = __hip_atomic_load(flags + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (b < ntiles) load_y(b);
  if (SKEW == 0 && partner < G && partner < ntiles) load_x(partner);  // round 0's consumed tile
  const uint32_t flag = wave_uniform(flagv);
  stamp(1);
  for (uint64_t i = 0; i < rounds + SKEW; ++i) {
    const uint64_t t = i * G + b;                           // packed this round (i < rounds)
    const uint64_t tp = (i - (uint64_t)SKEW) * G + partner;  // consumed this round (i >= SKEW)
    const bool pack = i < rounds && t < ntiles;
    const bool consume = i >= (uint64_t)SKEW && partner < G && tp < ntiles;
    if (consume && (SKEW > 0 || i > 0)) load_x(tp);
    // ---- pack: payload -> LDS -> packet-major stores (packets j and 64 + j of each 1 KiB chunk)
    if (pack) {
#pragma unroll
      for (int k = 0; k < U; ++k) *(u32x4*)&ldsP[wave][k][lane * 16] = yw[k];
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const uint64_t c = chunk(t, k);
        const auto rp = make_rsrc(pkts + 2 * c);
        const u32x2 lo = *(const u32x2*)&ldsP[wave][k][lane * 8];
        const u32x2 hi = *(const u32x2*)&ldsP[wave][k][512 + lane * 8];
        if (c + lane * 8 < bytes) store16<kSystem>(rp, lane * 16, LL16Packet::make(lo.x, lo.y, flag));
        if (c + 512 + lane * 8 < bytes) store16<kSystem>(rp, 1024 + lane * 16, LL16Packet::make(hi.x, hi.y, flag));
      }
      stamp(2);
      if (t + G < ntiles) load_y(t + G);
    }
    // ---- consume a partner tile: packet-major polls -> LDS -> payload-major sum and store
    if (consume) {
      // every poll of the tile issued before any is looked at (a readiness test right after each
      // load made the compiler wait for it before issuing the next).  Lanes past the end of the
      // buffer re-read the chunk's first packet (ignored); a chunk wholly past the end (uniform)
      // loads through a zero-length resource: out of range, zeros, no memory access.
      u32x4 v[2 * U];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const uint64_t c = cchunk(tp, k);
        const auto rp = __builtin_amdgcn_make_buffer_rsrc(pkts + 2 * c, 0, c < bytes ? 0xFFFFFFFFu : 0u, 0x00020000);
        v[2 * k] = load16<kSystem>(rp, c + lane * 8 < bytes ? lane * 16 : 0u);
        v[2 * k + 1] = load16<kSystem>(rp, c + 512 + lane * 8 < bytes ? 1024 + lane * 16 : 0u);
      }
      bool ok = true;
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const uint64_t c = cchunk(tp, k);
        if (c + lane * 8 < bytes) ok &= LL16Packet::ready(v[2 * k], flag);
        if (c + 512 + lane * 8 < bytes) ok &= LL16Packet::ready(v[2 * k + 1], flag);
      }
      if constexpr (COUNT) {
        uint32_t miss = 0;
#pragma unroll
        for (int i2 = 0; i2 < 2 * U; ++i2) {
          const uint64_t c = cchunk(tp, i2 / 2);
          if (c + (i2 & 1) * 512 + lane * 8 < bytes && !LL16Packet::ready(v[i2], flag)) ++miss;
        }
        // wave-wide sum of the misses, one atomic per wave
        for (int off = 32; off > 0; off >>= 1) miss += __shfl_xor(miss, off, 64);
        if (lane == 0 && miss) __hip_atomic_fetch_add(pollMiss, miss, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (!ok) {
#pragma unroll
        for (int i2 = 0; i2 < 2 * U; ++i2) {
          const uint64_t c = cchunk(tp, i2 / 2);
          const uint32_t off = (i2 & 1) * 1024 + lane * 16;
          if (c + (i2 & 1) * 512 + lane * 8 < bytes && !LL16Packet::ready(v[i2], flag)) {
            const auto rp = make_rsrc(pkts + 2 * c);
            SpinGuard g(budget);
            do {
              v[i2] = load16<kSystem>(rp, off);
              if (g.expired()) {
                report_packet_timeout(err, flag, 2 * c + off, v[i2].y != flag ? v[i2].y : v[i2].w);
                break;
              }
            } while (!LL16Packet::ready(v[i2], flag));
          }
        }
      }
      stamp(3);
#pragma unroll
      for (int k = 0; k < U; ++k) {
        *(u32x2*)&ldsC[wave][k][lane * 8] = u32x2{v[2 * k].x, v[2 * k].z};
        *(u32x2*)&ldsC[wave][k][512 + lane * 8] = u32x2{v[2 * k + 1].x, v[2 * k + 1].z};
      }
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const uint64_t c = cchunk(tp, k);
        const u32x4 p = *(const u32x4*)&ldsC[wave][k][lane * 16];
        if (c + lane * 16 < bytes) store16<LP>(make_rsrc(out + c), lane * 16, reduce4<DT, OP>(a[k], p));
      }
      stamp(4);
    }
    __builtin_amdgcn_wave_barrier();
  }
  bump_flags(flags, flag);
  stamp(5);
}

// Launch shape of the product kernel for `bytes` (nblocks > 0: the caller's grid), from the
// same-process shape sweeps (tools/sweep_self_reduce.py, profiles/r3_sweep_self_reduce.json), and
// since round 4 the one-round forms' hand-off partner from tools/small_bucket_probe.py
// (profiles/r4_small_bucket_probe*.json): in one round a workgroup's waves hand their packets to
// each other (wave w consumes wave w ^ 1's, same CU) instead of to workgroup b ^ 1 on another XCD.
// The packets still go through the packet buffer in memory with their flags polled; what goes away
// is the wait for a partner workgroup that the dispatcher started up to ~0.6 us later on another
// XCD: 64-256 KiB 3.44-3.46 against 4.04-4.12 us, 1 MiB 3.40 / 4.57, 2 MiB 4.11 / 5.93, 4 MiB
// 6.2 / 8.1 (graph-captured, one box).  The shape rule below (current since round 4):
// 4 waves x 1 KiB per workgroup and round, one workgroup per 4 KiB tile up to 1024 workgroups (4 per
// CU, all resident); 8 waves per workgroup for 1-4 MiB.  In every form the partner is the same
// workgroup's neighbouring wave (PMASK 0).
//  * one round (up to 4 MiB): unskewed, payload read and written with the default cache policy (a
//    bucket just written or read by the caller is served from the caches);
//  * 2-7 rounds: the partner's tile is consumed one round late (skew 1); from 8 rounds (48 MiB: 12)
//    two rounds late (skew 2); nt payload accesses.  The skew gives a packet time to land before its
//    first poll.
// Superseded round-3 figures (cross-XCD partner workgroup b ^ 1, two rounds unskewed): 3.6-3.7 us at
// 64-256 KiB; at 48 MiB 2.7 % of the packets missed their first poll with skew 2 (6.6 % with one,
// 13.9 % with none).
struct SelfReduceShape {
  int waves, units, nblocks;
  int skew;    // rounds between packing a tile and its partner consuming it
  bool plain;  // default-policy payload accesses (one round)
};
static SelfReduceShape selfReduceShape(uint64_t bytes, int nblocks) {
  SelfReduceShape sh{};
  sh.units = 1;
  if (nblocks <= 0 && bytes > (1u << 20) && bytes <= (4u << 20)) {
    // 1-4 MiB: one round of 8-wave workgroups (8 KiB tiles, at most 512 of them) -- half as many
    // workgroups to dispatch as 4-wave ones: 2 MiB 5.76 against 5.95 us, 3 MiB 7.0 / 7.25,
    // 4 MiB 7.95 / 8.43 (profiles/r3l_sweep_self_reduce_1_8MiB.json); at 1 MiB the 4-wave form is
    // ahead (4.53 / 4.76), from 6 MiB they are even
    sh.waves = 8;
    const uint64_t tiles8 = (bytes + 8191) / 8192;
    sh.nblocks = (int)tiles8 + (int)(tiles8 % 2);
    sh.skew = 0;
    sh.plain = true;
    return sh;
  }
  sh.waves = 4;
  const uint64_t tiles = (bytes + 4095) / 4096;
  sh.nblocks = nblocks > 0 ? nblocks : (int)(tiles < 1024 ? tiles : 1024);
  if (sh.nblocks % 2) sh.nblocks += 1;
  const uint64_t rounds = (tiles + sh.nblocks - 1) / sh.nblocks;
  // the partner is the neighbouring wave of the same workgroup in every form; with two or more rounds
  // its tile is consumed a round late (two from 8 rounds): 8 MiB 10.6 against 13.1 us (the cross-XCD
  // partner workgroup, unskewed), 16 MiB 19.4-19.5 / 21.9, 32-48 MiB even
  // (profiles/r4a_multi_round_probe.json)
  sh.skew = rounds >= 8 ? 2 : rounds >= 2 ? 1 : 0;
  sh.plain = rounds == 1;
  return sh;
}

template <int DT, int OP, int W, int U, int SKEW, bool COUNT, int LP = kNonTemporal, int PMASK = 1, bool TR = false>
static void launchSelfReduceShape(const void* x, const void* y, void* pkts, void* out, uint64_t bytes, uint32_t* flags,
                                  int nblocks, uint64_t budget, uint32_t* err, uint32_t* pollMiss, hipStream_t stream) {
  hipLaunchKernelGGL((selfReduceLL16LdsKernel<DT, OP, W, U, SKEW, COUNT, LP, PMASK, TR>), dim3(nblocks), dim3(64 * W), 0,
                     stream,
                     (const uint8_t*)x, (const uint8_t*)y, (uint8_t*)pkts, (uint8_t*)out, bytes, flags, budget, err,
                     pollMiss);
}

template <int DT, int OP>
static void launchSelfReduce(const void* x, const void* y, void* pkts, void* out, uint64_t bytes, uint32_t* flags,
                             int nblocks, uint64_t budget, uint32_t* err, hipStream_t stream) {
  const SelfReduceShape sh = selfReduceShape(bytes, nblocks);
  // wave w of a workgroup consumes what wave w ^ 1 of the same workgroup packed (PMASK 0)
  if (sh.waves == 8)
    launchSelfReduceShape<DT, OP, 8, 1, 0, false, kPlain, 0>(x, y, pkts, out, bytes, flags, sh.nblocks, budget, err,
                                                                 nullptr, stream);
  else if (sh.plain)
    launchSelfReduceShape<DT, OP, 4, 1, 0, false, kPlain, 0>(x, y, pkts, out, bytes, flags, sh.nblocks, budget, err,
                                                                 nullptr, stream);
  else if (sh.skew == 2)
    launchSelfReduceShape<DT, OP, 4, 1, 2, false, kNonTemporal, 0>(x, y, pkts, out, bytes, flags, sh.nblocks, budget,
                                                                   err, nullptr, stream);
  else if (sh.skew == 1)
    launchSelfReduceShape<DT, OP, 4, 1, 1, false, kNonTemporal, 0>(x, y, pkts, out, bytes, flags, sh.nblocks, budget,
                                                                   err, nullptr, stream);
  else  // a caller's grid with more workgroups than tiles
    launchSelfReduceShape<DT, OP, 4, 1, 0, false, kNonTemporal, 0>(x, y, pkts, out, bytes, flags, sh.nblocks, budget,
                                                                   err, nullptr, stream);
}

// Streaming copy (read S, write S) used by the benchmark to measure the achievable HBM ceiling on
// the same box in the same run.
template <int U>
__global__ void __launch_bounds__(256) copyKernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                  uint64_t nunits) {
  const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
  for (uint64_t u0 = (uint64_t)blockIdx.x * 256 * U; u0 < nunits; u0 += stride) {
    auto rs = make_rsrc(src + u0 * 16);
    auto rd = make_rsrc(dst + u0 * 16);
    u32x4 w[U];
#pragma unroll
    for (int k = 0; k < U; ++k)
      if (u0 + k * 256 + threadIdx.x < nunits) w[k] = load16<kNonTemporal>(rs, (k * 256 + threadIdx.x) * 16);
#pragma unroll
    for (int k = 0; k < U; ++k)
      if (u0 + k * 256 + threadIdx.x < nunits) store16<kNonTemporal>(rd, (k * 256 + threadIdx.x) * 16, w[k]);
  }
}

// Same-traffic streaming ceiling of the self-reduce (benchmark only): the large form's exact memory
// accesses -- per wave and round, 1 KiB of Y read, 2 KiB of packets stored packet-major (two 1 KiB
// instructions, system scope), the partner wave's 2 KiB of packets from two rounds earlier read (system
// scope), 1 KiB of X read and 1 KiB of O written, all on the same buffers, grid and rounds -- with no
// flags, readiness tests, re-polls or LDS.  Its time is what the memory system gives this 7*S access
// mix; the product kernel's time against it is the cost of the hand-off itself.  (The packets read
// are whatever is there: the output is meaningless.)
__global__ void __launch_bounds__(256) selfReduceStreamKernel(const uint8_t* __restrict__ x, const uint8_t* __restrict__ y,
                                                              uint8_t* pkts, uint8_t* __restrict__ out, uint64_t bytes) {
  constexpr uint64_t kTile = 4096;  // 4 waves x 1 KiB
  const uint32_t G = gridDim.x, b = blockIdx.x;
  const uint32_t wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  const uint64_t ntiles = bytes / kTile;
  const uint64_t rounds = (ntiles + G - 1) / G;
  for (uint64_t i = 0; i < rounds; ++i) {
    const uint64_t t = i * G + b;
    if (t >= ntiles) break;
    // the product's partner (round 4): wave ^ 1 of the same workgroup, its tile two rounds late
    const uint64_t tp = ((i >= 2 ? i - 2 : i + rounds - 2) * G + b) % ntiles;
    const uint64_t c = t * kTile + wave * 1024, cp = tp * kTile + (wave ^ 1u) * 1024;
    const u32x4 yv = load16<kNonTemporal>(make_rsrc(y + c), lane * 16);
    const u32x4 xv = load16<kNonTemporal>(make_rsrc(x + cp), lane * 16);
    const auto rpp = make_rsrc(pkts + 2 * cp);
    const u32x4 p0 = load16<kSystem>(rpp, lane * 16);
    const u32x4 p1 = load16<kSystem>(rpp, 1024 + lane * 16);
    const auto rp = make_rsrc(pkts + 2 * c);
    store16<kSystem>(rp, lane * 16, u32x4{yv.x, 0u, yv.y, 0u});  // flag 0: no call ever waits for it
    store16<kSystem>(rp, 1024 + lane * 16, u32x4{yv.z, 0u, yv.w, 0u});
    store16<kNonTemporal>(make_rsrc(out + cp), lane * 16, u32x4{xv.x ^ p0.x, xv.y ^ p0.z, xv.z ^ p1.x, xv.w ^ p1.z});
  }
}

// An independent ceiling for the same 4:3 read:write mix (benchmark only): none of the self-reduce's
// choices -- a grid-stride loop over 16-byte units, 2048 workgroups of 256 lanes, U units per lane in
// flight, every access non-temporal; per unit X, Y and two packet units read from `pin`, two units
// written to a separate `pout` and one to `out` (4 * bytes read, 3 * bytes written, no buffer read
// and written in the same launch).
template <int U>
__global__ void __launch_bounds__(256) mixStreamKernel(const uint8_t* __restrict__ x, const uint8_t* __restrict__ y,
                                                       const uint8_t* __restrict__ pin, uint8_t* __restrict__ pout,
                                                       uint8_t* __restrict__ out, uint64_t nunits) {
  // a workgroup's pass covers 256 * U units of X / Y / out and the 512 * U units of pin / pout at twice
  // their offset; every wave instruction touches 1 KiB of contiguous, whole lines
  const uint64_t step = (uint64_t)gridDim.x * 256 * U;
  for (uint64_t base = (uint64_t)blockIdx.x * 256 * U; base < nunits; base += step) {
    u32x4 a[U], b[U], p0[U], p1[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint64_t u = base + (uint64_t)k * 256 + threadIdx.x, q = 2 * (base + (uint64_t)k * 256) + threadIdx.x;
      if (u < nunits) {
        a[k] = load16<kNonTemporal>(make_rsrc(x), (uint32_t)(u * 16));
        b[k] = load16<kNonTemporal>(make_rsrc(y), (uint32_t)(u * 16));
        p0[k] = load16<kNonTemporal>(make_rsrc(pin), (uint32_t)(q * 16));
        p1[k] = load16<kNonTemporal>(make_rsrc(pin), (uint32_t)((q + 256) * 16));
      }
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint64_t u = base + (uint64_t)k * 256 + threadIdx.x, q = 2 * (base + (uint64_t)k * 256) + threadIdx.x;
      if (u < nunits) {
        store16<kNonTemporal>(make_rsrc(pout), (uint32_t)(q * 16), u32x4{b[k].x, 0u, b[k].y, 0u});
        store16<kNonTemporal>(make_rsrc(pout), (uint32_t)((q + 256) * 16), u32x4{b[k].z, 0u, b[k].w, 0u});
        store16<kNonTemporal>(make_rsrc(out), (uint32_t)(u * 16),
                              u32x4{a[k].x ^ p0[k].x, a[k].y ^ p0[k].z, a[k].z ^ p1[k].x, a[k].w ^ p1[k].z});
      }
    }
  }
}

// Several independent copies in ONE launch: workgroups [j*B, (j+1)*B) move job j.  The xGMI probe
// uses it so that all peers' links are driven by one kernel on one stream (one hardware queue),
// instead of one stream per peer that the pool's GPU_MAX_HW_QUEUES=4 would serialise.  Remote
// sides are IPC-mapped peer memory: loads and stores of the remote side are system scope.
struct CopyJobs {
  const uint8_t* src[MSCCLPP_AMD_MAX_RANKS * 2];
  uint8_t* dst[MSCCLPP_AMD_MAX_RANKS * 2];
  uint64_t units[MSCCLPP_AMD_MAX_RANKS * 2];
};

template <int U, int LP = kSystem, int SP = kSystem>
__global__ void __launch_bounds__(256) copyJobsKernel(CopyJobs jobs, uint32_t blocksPerJob) {
  const uint32_t j = blockIdx.x / blocksPerJob, jb = blockIdx.x % blocksPerJob;
  const uint8_t* src = jobs.src[j];
  uint8_t* dst = jobs.dst[j];
  const uint64_t nunits = jobs.units[j];
  const uint64_t stride = (uint64_t)blocksPerJob * 256 * U;
  for (uint64_t u0 = (uint64_t)jb * 256 * U; u0 < nunits; u0 += stride) {
    auto rs = make_rsrc(src + u0 * 16);
    auto rd = make_rsrc(dst + u0 * 16);
    u32x4 w[U];
#pragma unroll
    for (int k = 0; k < U; ++k)
      if (u0 + k * 256 + threadIdx.x < nunits) w[k] = load16<LP>(rs, (k * 256 + threadIdx.x) * 16);
#pragma unroll
    for (int k = 0; k < U; ++k)
      if (u0 + k * 256 + threadIdx.x < nunits) store16<SP>(rd, (k * 256 + threadIdx.x) * 16, w[k]);
  }
}

}  // namespace mscclpp_amd

using namespace mscclpp_amd;

#ifdef MSCCLPP_AMD_DIAG
// Tuning / diagnostic entry (fp16 SUM), built only into the test diagnostics library
// (tests/bin/libselfreduce_diag.so, mscclpp_amd/_build.py build_diag): any (waves, units, skew depth
// 0 / 1, or 2 for 4 waves) shape on any grid, and with count bit 0 the number of packets whose first
// poll missed added to pollMiss[0] (must not be null).
extern "C" int mscclppAmdSelfReduceLL16Shape(const void* x, const void* y, void* pkts, void* out, size_t bytes,
                                             uint32_t* flags, int nblocks, int waves, int units, int skew, int count,
                                             uint64_t budgetTicks, uint32_t* err, uint32_t* pollMiss, void* streamPtr) {
  hipStream_t s = (hipStream_t)streamPtr;
  if (!x || !y || !pkts || !out || !flags || bytes == 0 || (bytes % 16) != 0 || nblocks <= 0 || nblocks > 4096) return 4;
  if ((count & 1) && !pollMiss) return 4;
  if (nblocks % 2) nblocks += 1;
  // count: bit 0 = count first-poll misses, bit 1 = default-policy payload loads / stores (the small
  // form's choice)
  const bool plain = (count & 2) != 0;
  const int pmask = (count & 4) ? 0 : (count & 8) ? 8 : 1;  // bit 2: partner wave w ^ 1 of the workgroup; bit 3: b ^ 8
  count &= 1;
  if (pmask != 1) {  // 4 x 1 KiB, 4 x 2 KiB or 8 x 1 KiB waves, nt payload, skew 0 / 1 / 2 (multi-round forms)
    if (count || plain || (pmask == 8 && nblocks % 16)) return 4;
#define SRPM(W, U, SK, PM)                                                                                        \
    if (waves == W && units == U && skew == SK && pmask == PM) {                                                  \
      launchSelfReduceShape<kF16, kSum, W, U, SK, false, kNonTemporal, PM>(x, y, pkts, out, bytes, flags, nblocks, \
                                                                          budgetTicks, err, pollMiss, s);          \
      return hipGetLastError() == hipSuccess ? 0 : 1;                                                             \
    }
    SRPM(4, 1, 0, 0) SRPM(4, 1, 1, 0) SRPM(4, 1, 2, 0) SRPM(4, 1, 0, 8) SRPM(4, 1, 1, 8) SRPM(4, 1, 2, 8)
    SRPM(4, 2, 1, 0) SRPM(4, 2, 2, 0) SRPM(8, 1, 1, 0) SRPM(8, 1, 2, 0)
#undef SRPM
    return 4;
  }
#define SRS(W, U, SK, C)                                                                                      \
  if (waves == W && units == U && skew == SK && (count != 0) == C) {                                          \
    if (plain)                                                                                                \
      launchSelfReduceShape<kF16, kSum, W, U, SK, C, kPlain>(x, y, pkts, out, bytes, flags, nblocks,          \
                                                             budgetTicks, err, pollMiss, s);                 \
    else                                                                                                      \
      launchSelfReduceShape<kF16, kSum, W, U, SK, C>(x, y, pkts, out, bytes, flags, nblocks, budgetTicks, err, \
                                                     pollMiss, s);                                           \
    return hipGetLastError() == hipSuccess ? 0 : 1;                                                           \
  }
#define SRS_SK(W, U) SRS(W, U, 1, false) SRS(W, U, 0, false) SRS(W, U, 1, true) SRS(W, U, 0, true)
  SRS_SK(1, 1) SRS_SK(2, 1) SRS_SK(2, 2) SRS_SK(4, 1) SRS_SK(4, 2) SRS_SK(8, 1) SRS_SK(8, 2)
  SRS(4, 1, 2, false) SRS(4, 1, 2, true) SRS(4, 2, 2, false) SRS(4, 2, 2, true)
#undef SRS_SK
#undef SRS
  return 4;
}

// Small-bucket probe (fp16 SUM, one round, default-policy payload): `waves` per workgroup on
// `nblocks` workgroups of one 1 KiB tile per wave, partners b ^ pmask (1 or 8; with 8 the grid must be
// a multiple of 16; 0: wave w ^ 1 of the same workgroup), trace != 0: phase stamps into `trace` (nblocks * 8 uint64).
extern "C" int mscclppAmdSelfReduceSmallProbe(const void* x, const void* y, void* pkts, void* out, size_t bytes,
                                              uint32_t* flags, int nblocks, int waves, int pmask, uint64_t* trace,
                                              uint64_t budgetTicks, uint32_t* err, void* streamPtr) {
  hipStream_t s = (hipStream_t)streamPtr;
  if (!x || !y || !pkts || !out || !flags || bytes == 0 || (bytes % 16) != 0 || nblocks <= 0 || nblocks > 1024) return 4;
  if ((uint64_t)nblocks * waves * 1024 < bytes) return 4;  // one round only
  if (pmask == 8 ? (nblocks % 16) != 0 : pmask == 0 ? waves < 2 : (pmask != 1 || nblocks % 2)) return 4;
  uint32_t* tr = (uint32_t*)trace;
#define SRP(W, PM, T)                                                                                          \
  if (waves == W && pmask == PM && (trace != nullptr) == T) {                                                 \
    launchSelfReduceShape<kF16, kSum, W, 1, 0, false, kPlain, PM, T>(x, y, pkts, out, bytes, flags, nblocks,   \
                                                                      budgetTicks, err, tr, s);                \
    return hipGetLastError() == hipSuccess ? 0 : 1;                                                           \
  }
#define SRP_W(W) SRP(W, 1, false) SRP(W, 1, true) SRP(W, 8, false) SRP(W, 8, true) SRP(W, 0, false) SRP(W, 0, true)
  SRP(1, 1, false) SRP(1, 1, true) SRP(1, 8, false) SRP(1, 8, true)
  SRP_W(2) SRP_W(4) SRP_W(8) SRP_W(16)
#undef SRP_W
#undef SRP
  return 4;
}
#endif

// The launch shape the product entry point picks for `bytes` with nblocks = 0 (tests, tools).
extern "C" int mscclppAmdSelfReduceLL16DefaultShape(size_t bytes, int* waves, int* units, int* nblocks, int* skew) {
  if (!waves || !units || !nblocks || !skew) return 4;
  const SelfReduceShape sh = selfReduceShape(bytes, 0);
  *waves = sh.waves;
  *units = sh.units;
  *nblocks = sh.nblocks;
  *skew = sh.skew;
  return 0;
}

extern "C" int mscclppAmdCopy(const void* src, void* dst, size_t bytes, int nblocks, void* streamPtr) {
  if (!src || !dst || bytes == 0 || (bytes % 16) != 0) return 4;
  if (nblocks <= 0) nblocks = 2048;
  hipLaunchKernelGGL((copyKernel<4>), dim3(nblocks), dim3(256), 0, (hipStream_t)streamPtr, (const uint8_t*)src,
                     (uint8_t*)dst, (uint64_t)(bytes / 16));
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

extern "C" int mscclppAmdCopyJobsPolicy(const void* const* srcs, void* const* dsts, const size_t* bytes, int njobs,
                                        int blocksPerJob, int loadPolicy, int storePolicy, void* streamPtr);

extern "C" int mscclppAmdSelfReduceStream(const void* x, const void* y, void* pkts, void* out, size_t bytes,
                                          void* streamPtr) {
  // the product's large-form grid: one workgroup per 4 KiB tile, at most 1024
  if (!x || !y || !pkts || !out || bytes == 0 || bytes % 8192) return 4;
  const uint64_t tiles = bytes / 4096;
  const int nblocks = (int)(tiles < 1024 ? tiles : 1024);
  hipLaunchKernelGGL(selfReduceStreamKernel, dim3(nblocks), dim3(256), 0, (hipStream_t)streamPtr, (const uint8_t*)x,
                     (const uint8_t*)y, (uint8_t*)pkts, (uint8_t*)out, (uint64_t)bytes);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

extern "C" int mscclppAmdMixStream(const void* x, const void* y, const void* pin, void* pout, void* out, size_t bytes,
                                   int nblocks, void* streamPtr) {
  // buffer offsets are 32-bit (buffer resources): pin / pout hold 2 * bytes
  // whole 4 KiB passes only: a pass's pin / pout units lie inside 2 * bytes exactly when it is whole
  if (!x || !y || !pin || !pout || !out || bytes == 0 || bytes % 4096 || 2 * (uint64_t)bytes > 0xFFFFFFF0ull) return 4;
  if (nblocks <= 0) nblocks = 2048;
  hipLaunchKernelGGL((mixStreamKernel<4>), dim3(nblocks), dim3(256), 0, (hipStream_t)streamPtr, (const uint8_t*)x,
                     (const uint8_t*)y, (const uint8_t*)pin, (uint8_t*)pout, (uint8_t*)out, (uint64_t)(bytes / 16));
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

extern "C" int mscclppAmdCopyJobs(const void* const* srcs, void* const* dsts, const size_t* bytes, int njobs,
                                  int blocksPerJob, void* streamPtr) {
  return mscclppAmdCopyJobsPolicy(srcs, dsts, bytes, njobs, blocksPerJob, 0, 0, streamPtr);
}

// The same copy with the cache policy of its loads / stores chosen (0 = sc0 sc1 system scope, the
// policy of every remote access in the collectives; 1 = plain; 2 = nt; 3 = sc1 agent scope): the
// xGMI probe measures what each policy delivers over the links.
extern "C" int mscclppAmdCopyJobsPolicy(const void* const* srcs, void* const* dsts, const size_t* bytes, int njobs,
                                        int blocksPerJob, int loadPolicy, int storePolicy, void* streamPtr) {
  if (loadPolicy < 0 || loadPolicy > 3 || storePolicy < 0 || storePolicy > 3) return 4;
  if (!srcs || !dsts || !bytes || njobs < 1 || njobs > 2 * MSCCLPP_AMD_MAX_RANKS) return 4;
  if (blocksPerJob <= 0) blocksPerJob = 128;
  if ((long)blocksPerJob * njobs > 65535) return 4;
  CopyJobs jobs{};
  for (int j = 0; j < njobs; ++j) {
    if (!srcs[j] || !dsts[j] || bytes[j] == 0 || bytes[j] % 16) return 4;
    jobs.src[j] = (const uint8_t*)srcs[j];
    jobs.dst[j] = (uint8_t*)dsts[j];
    jobs.units[j] = bytes[j] / 16;
  }
  const dim3 grid(blocksPerJob * njobs), block(256);
  hipStream_t st = (hipStream_t)streamPtr;
  const uint32_t bpj = (uint32_t)blocksPerJob;
  auto go = [&](auto kern) { hipLaunchKernelGGL(kern, grid, block, 0, st, jobs, bpj); };
  switch (loadPolicy * 4 + storePolicy) {  // loads of remote data: system or plain; stores: any
    case 0: go(copyJobsKernel<4, kSystem, kSystem>); break;
    case 1: go(copyJobsKernel<4, kSystem, kPlain>); break;
    case 2: go(copyJobsKernel<4, kSystem, kNonTemporal>); break;
    case 3: go(copyJobsKernel<4, kSystem, kAgent>); break;
    case 4: go(copyJobsKernel<4, kPlain, kSystem>); break;
    case 5: go(copyJobsKernel<4, kPlain, kPlain>); break;
    case 8: go(copyJobsKernel<4, kNonTemporal, kSystem>); break;
    case 12: go(copyJobsKernel<4, kAgent, kSystem>); break;
    default: return 4;
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

extern "C" int mscclppAmdSelfReduceLL16(const void* x, const void* y, void* pkts, void* out, size_t bytes, int dtype,
                                        int op, uint32_t* flags, int nblocks, uint64_t budgetTicks, uint32_t* err,
                                        void* streamPtr) {
  hipStream_t stream = (hipStream_t)streamPtr;
  if (!x || !y || !pkts || !out || !flags || bytes == 0 || (bytes % 16) != 0) return 4;
  if ((uintptr_t)flags % 16) return 4;  // the flag slots above the grid are refreshed 16 bytes at a time
  // nblocks <= 0: the default shape (selfReduceShape); otherwise the large form on that grid, at most
  // 1024 workgroups = 4 per CU (16 KiB LDS each), all resident, so every partner pair is co-resident
  if (nblocks > 1024) return 4;
  MSCCLPP_AMD_DISPATCH_ALL(dtype, op, launchSelfReduce, x, y, pkts, out, (uint64_t)bytes, flags, nblocks, budgetTicks, err, stream);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
