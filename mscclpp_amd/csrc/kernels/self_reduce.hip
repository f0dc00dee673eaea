// 1-GPU LL16 self-reduce microbench (BASELINE.json configs[1]).
//
//   P = LL16(Y, flag)                 pack   (copyToPackets<LL16>, copy_device.hpp:160-171)
//   O = X (op) unpack(P, flag)        reduce (LL16Packet::read + calVectorAccum, allreduce_packet.cu:93-108)
//
// One launch, two roles per workgroup.  Workgroup b packs tile t = i*G + b and then consumes the
// tile packed by its partner b^1 in the same round, so every packet is handed from one CU to a CU
// on a different XCD (blocks are dealt round-robin over the 8 XCDs) purely through the LL flags,
// exactly as a peer GPU's packets arrive in the AllReduce.  Partners progress in lock-step, so the
// only residency requirement is that both workgroups of a pair are resident: the host keeps the
// grid at or below 4 workgroups per CU (256 CUs).  Every spin is time-bounded.
//
// Algorithmic HBM bytes per launch: 7*S (Y read S, P written 2S, P read 2S, X read S, O written S).
#include "common.hpp"

namespace mscclpp_amd {

template <int DT, int OP, int U, int PKT_POLICY, int LD_POLICY = kSystem>
__global__ void __launch_bounds__(256) selfReduceLL16Kernel(const uint8_t* __restrict__ x, const uint8_t* __restrict__ y,
                                                            uint8_t* pkts, uint8_t* __restrict__ out,
                                                            uint64_t nunits, uint32_t* flags, uint64_t budget,
                                                            uint32_t* err) {
  constexpr uint32_t kThreads = 256;
  constexpr uint64_t kTileUnits = (uint64_t)kThreads * U;
  const uint32_t G = gridDim.x;
  const uint32_t b = blockIdx.x;
  const uint32_t tid = threadIdx.x;
  const uint32_t flag = flags[b];
  const uint64_t ntiles = (nunits + kTileUnits - 1) / kTileUnits;
  const uint32_t partner = b ^ 1u;

  // Software pipeline per round: the X loads of the tile to consume and the Y loads of the NEXT
  // tile to pack are in flight while this round's packets are stored and the partner's packets
  // are polled, so every phase keeps loads outstanding.
  u32x4 yw[U];
  auto load_y = [&](uint64_t t) {
    const uint64_t u0 = t * kTileUnits;
    auto ry = make_rsrc(y + u0 * 16);
#pragma unroll
    for (int k = 0; k < U; ++k)
      if (u0 + k * kThreads + tid < nunits) yw[k] = load16<kNonTemporal>(ry, (uint32_t)((k * kThreads + tid) * 16));
  };
  if (b < ntiles) load_y(b);
  for (uint64_t base = 0; base < ntiles; base += G) {
    const uint64_t t = base + b;
    const uint64_t tp = base + partner;
    const bool consume = partner < G && tp < ntiles;
    u32x4 a[U];
    if (consume) {
      const uint64_t u0 = tp * kTileUnits;
      auto rx = make_rsrc(x + u0 * 16);
#pragma unroll
      for (int k = 0; k < U; ++k)
        if (u0 + k * kThreads + tid < nunits) a[k] = load16<kNonTemporal>(rx, (uint32_t)((k * kThreads + tid) * 16));
    }
    // ---- pack my tile, then prefetch the next one
    if (t < ntiles) {
      const uint64_t u0 = t * kTileUnits;
      auto rp = make_rsrc(pkts + u0 * 32);
#pragma unroll
      for (int k = 0; k < U; ++k)
        if (u0 + k * kThreads + tid < nunits) ll16_put_unit<PKT_POLICY>(rp, (uint32_t)((k * kThreads + tid) * 32), yw[k], flag);
      if (t + G < ntiles) load_y(t + G);
    }
    // ---- consume my partner's tile
    if (consume) {
      const uint64_t u0 = tp * kTileUnits;
      auto ro = make_rsrc(out + u0 * 16);
      auto rp = make_rsrc(pkts + u0 * 32);
      u32x4 v[U];
      bool ok = true;
#pragma unroll
      for (int k = 0; k < U; ++k)
        if (u0 + k * kThreads + tid < nunits) ok &= ll16_try_unit<LD_POLICY>(rp, (uint32_t)((k * kThreads + tid) * 32), flag, v[k]);
      if (!ok) {
#pragma unroll
        for (int k = 0; k < U; ++k)
          if (u0 + k * kThreads + tid < nunits)
            v[k] = ll16_get_unit<LD_POLICY>(rp, (uint32_t)((k * kThreads + tid) * 32), flag, budget, err);
      }
#pragma unroll
      for (int k = 0; k < U; ++k)
        if (u0 + k * kThreads + tid < nunits)
          store16<kNonTemporal>(ro, (uint32_t)((k * kThreads + tid) * 16), reduce4<DT, OP>(a[k], v[k]));
    }
  }
  bump_flags(flags, flag);
}

// Packet-major lane mapping: lane m of a wave owns LL16 packet m, so every packet store and poll is
// one contiguous 1 KiB wave instruction (whole 64-byte lines), and the payload side moves 8 bytes
// per lane (512 B contiguous per instruction).  The payload-major form above writes each packet
// line in two halves from two instructions; on gfx950 WRITE_SIZE shows those partial-line stores
// cost a full line each (5*S written instead of 3*S).
template <int DT, int OP, int U, int PKT_POLICY, int LD_POLICY = kSystem>
__global__ void __launch_bounds__(256) selfReduceLL16PmKernel(const uint8_t* __restrict__ x, const uint8_t* __restrict__ y,
                                                              uint8_t* pkts, uint8_t* __restrict__ out,
                                                              uint64_t npkts, uint32_t* flags, uint64_t budget,
                                                              uint32_t* err) {
  constexpr uint32_t kThreads = 256;
  constexpr uint64_t kTilePkts = (uint64_t)kThreads * U;
  const uint32_t G = gridDim.x;
  const uint32_t b = blockIdx.x;
  const uint32_t tid = threadIdx.x;
  const uint32_t flag = flags[b];
  const uint64_t ntiles = (npkts + kTilePkts - 1) / kTilePkts;
  const uint32_t partner = b ^ 1u;
  u32x2 yw[U];
  auto load_y = [&](uint64_t t) {
    const uint64_t p0 = t * kTilePkts;
    auto ry = make_rsrc(y + p0 * 8);
#pragma unroll
    for (int k = 0; k < U; ++k)
      if (p0 + k * kThreads + tid < npkts) yw[k] = load8<kNonTemporal>(ry, (uint32_t)((k * kThreads + tid) * 8));
  };
  if (b < ntiles) load_y(b);
  for (uint64_t base = 0; base < ntiles; base += G) {
    const uint64_t t = base + b;
    const uint64_t tp = base + partner;
    const bool consume = partner < G && tp < ntiles;
    u32x2 a[U];
    if (consume) {
      const uint64_t p0 = tp * kTilePkts;
      auto rx = make_rsrc(x + p0 * 8);
#pragma unroll
      for (int k = 0; k < U; ++k)
        if (p0 + k * kThreads + tid < npkts) a[k] = load8<kNonTemporal>(rx, (uint32_t)((k * kThreads + tid) * 8));
    }
    if (t < ntiles) {
      const uint64_t p0 = t * kTilePkts;
      auto rp = make_rsrc(pkts + p0 * 16);
#pragma unroll
      for (int k = 0; k < U; ++k)
        if (p0 + k * kThreads + tid < npkts)
          store16<PKT_POLICY>(rp, (uint32_t)((k * kThreads + tid) * 16), LL16Packet::make(yw[k].x, yw[k].y, flag));
      if (t + G < ntiles) load_y(t + G);
    }
    if (consume) {
      const uint64_t p0 = tp * kTilePkts;
      auto ro = make_rsrc(out + p0 * 8);
      auto rp = make_rsrc(pkts + p0 * 16);
      u32x4 v[U];
      bool ok = true;
#pragma unroll
      for (int k = 0; k < U; ++k)
        if (p0 + k * kThreads + tid < npkts) {
          v[k] = load16<LD_POLICY>(rp, (uint32_t)((k * kThreads + tid) * 16));
          ok &= LL16Packet::ready(v[k], flag);
        }
      if (!ok) {
#pragma unroll
        for (int k = 0; k < U; ++k) {
          if (p0 + k * kThreads + tid < npkts && !LL16Packet::ready(v[k], flag)) {
            SpinGuard g(budget);
            do {
              v[k] = load16<LD_POLICY>(rp, (uint32_t)((k * kThreads + tid) * 16));
              if (g.expired()) {
                report_error(err, kErrPacketTimeout);
                break;
              }
            } while (!LL16Packet::ready(v[k], flag));
          }
        }
      }
#pragma unroll
      for (int k = 0; k < U; ++k)
        if (p0 + k * kThreads + tid < npkts) {
          u32x2 r;
          r.x = reduce_word<DT, OP>(a[k].x, v[k].x);
          r.y = reduce_word<DT, OP>(a[k].y, v[k].z);
          store8<kNonTemporal>(ro, (uint32_t)((k * kThreads + tid) * 8), r);
        }
    }
  }
  bump_flags(flags, flag);
}

// LDS-staged packets: the payload side moves 16 bytes per lane (one dwordx4 per wave instruction,
// 1 KiB per wave) and the packet side stays packet-major (lane j owns packet j).  A wave turns its
// 1 KiB of payload into 128 packets through 1 KiB of its own LDS: each lane writes its 16 bytes, then
// reads back the 8 bytes of packet j and of packet 64 + j; the consumer runs the same swizzle in
// reverse before the 16-byte-per-lane sum and output store.  LDS traffic per wave-tile is three
// ds ops per side; the crossing stays inside one wave, so no barrier is needed (one wave's LDS
// operations complete in order).
template <int DT, int OP, int U>
__global__ void __launch_bounds__(256) selfReduceLL16LdsKernel(const uint8_t* __restrict__ x, const uint8_t* __restrict__ y,
                                                               uint8_t* pkts, uint8_t* __restrict__ out, uint64_t bytes,
                                                               uint32_t* flags, uint64_t budget, uint32_t* err) {
  constexpr uint32_t kWaves = 4;
  constexpr uint64_t kTileBytes = (uint64_t)kWaves * U * 1024;  // payload bytes per workgroup and round
  __shared__ __attribute__((aligned(16))) uint8_t lds[kWaves][U][1024];
  const uint32_t G = gridDim.x, b = blockIdx.x;
  const uint32_t wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  const uint32_t flag = flags[b];
  const uint64_t ntiles = (bytes + kTileBytes - 1) / kTileBytes;
  const uint32_t partner = b ^ 1u;
  // payload byte offset of (tile, sub-tile k) for this wave: 1 KiB chunks dealt k-major over waves
  auto chunk = [&](uint64_t t, int k) { return t * kTileBytes + (uint64_t)(k * kWaves + wave) * 1024; };
  u32x4 yw[U];
  auto load_y = [&](uint64_t t) {
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint64_t c = chunk(t, k);
      if (c + lane * 16 < bytes) yw[k] = load16<kNonTemporal>(make_rsrc(y + c), lane * 16);
    }
  };
  if (b < ntiles) load_y(b);
  for (uint64_t base = 0; base < ntiles; base += G) {
    const uint64_t t = base + b;
    const uint64_t tp = base + partner;
    const bool consume = partner < G && tp < ntiles;
    u32x4 a[U];
    if (consume) {
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const uint64_t c = chunk(tp, k);
        if (c + lane * 16 < bytes) a[k] = load16<kNonTemporal>(make_rsrc(x + c), lane * 16);
      }
    }
    // ---- pack: payload -> LDS -> packet-major stores (packets j and 64 + j of each 1 KiB chunk)
    if (t < ntiles) {
#pragma unroll
      for (int k = 0; k < U; ++k) *(u32x4*)&lds[wave][k][lane * 16] = yw[k];
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const uint64_t c = chunk(t, k);
        const auto rp = make_rsrc(pkts + 2 * c);
        const u32x2 lo = *(const u32x2*)&lds[wave][k][lane * 8];
        const u32x2 hi = *(const u32x2*)&lds[wave][k][512 + lane * 8];
        if (c + lane * 8 < bytes) store16<kSystem>(rp, lane * 16, LL16Packet::make(lo.x, lo.y, flag));
        if (c + 512 + lane * 8 < bytes) store16<kSystem>(rp, 1024 + lane * 16, LL16Packet::make(hi.x, hi.y, flag));
      }
      __builtin_amdgcn_wave_barrier();
      if (t + G < ntiles) load_y(t + G);
    }
    // ---- consume my partner's tile: packet-major polls -> LDS -> payload-major sum and store
    if (consume) {
      u32x4 v[2 * U];
      bool ok = true;
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const uint64_t c = chunk(tp, k);
        const auto rp = make_rsrc(pkts + 2 * c);
        if (c + lane * 8 < bytes) {
          v[2 * k] = load16<kSystem>(rp, lane * 16);
          ok &= LL16Packet::ready(v[2 * k], flag);
        }
        if (c + 512 + lane * 8 < bytes) {
          v[2 * k + 1] = load16<kSystem>(rp, 1024 + lane * 16);
          ok &= LL16Packet::ready(v[2 * k + 1], flag);
        }
      }
      if (!ok) {
#pragma unroll
        for (int i = 0; i < 2 * U; ++i) {
          const uint64_t c = chunk(tp, i / 2);
          const uint32_t off = (i & 1) * 1024 + lane * 16;
          if (c + (i & 1) * 512 + lane * 8 < bytes && !LL16Packet::ready(v[i], flag)) {
            const auto rp = make_rsrc(pkts + 2 * c);
            SpinGuard g(budget);
            do {
              v[i] = load16<kSystem>(rp, off);
              if (g.expired()) {
                report_error(err, kErrPacketTimeout);
                break;
              }
            } while (!LL16Packet::ready(v[i], flag));
          }
        }
      }
#pragma unroll
      for (int k = 0; k < U; ++k) {
        *(u32x2*)&lds[wave][k][lane * 8] = u32x2{v[2 * k].x, v[2 * k].z};
        *(u32x2*)&lds[wave][k][512 + lane * 8] = u32x2{v[2 * k + 1].x, v[2 * k + 1].z};
      }
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const uint64_t c = chunk(tp, k);
        const u32x4 p = *(const u32x4*)&lds[wave][k][lane * 16];
        if (c + lane * 16 < bytes) store16<kNonTemporal>(make_rsrc(out + c), lane * 16, reduce4<DT, OP>(a[k], p));
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  bump_flags(flags, flag);
}

template <int DT, int OP>
static void launchSelfReduce(const void* x, const void* y, void* pkts, void* out, uint64_t bytes, uint32_t* flags,
                             int nblocks, uint64_t budget, uint32_t* err, hipStream_t stream) {
  // LDS-staged packets, 2 KiB of payload per wave and round (tools/sweep_self_reduce.py: 56.3-57.3 us
  // at 48 MiB and 1024 workgroups vs 57.7-58.9 us for the packet-major register form, variant 13)
  hipLaunchKernelGGL((selfReduceLL16LdsKernel<DT, OP, 2>), dim3(nblocks), dim3(256), 0, stream, (const uint8_t*)x,
                     (const uint8_t*)y, (uint8_t*)pkts, (uint8_t*)out, bytes, flags, budget, err);
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

}  // namespace mscclpp_amd

using namespace mscclpp_amd;

// Tuning entry (fp16 SUM): variant selects <U, packet store policy, packet load policy>.
extern "C" int mscclppAmdSelfReduceLL16Variant(const void* x, const void* y, void* pkts, void* out, size_t bytes,
                                               uint32_t* flags, int nblocks, int variant, uint64_t budgetTicks,
                                               uint32_t* err, void* streamPtr) {
  hipStream_t s = (hipStream_t)streamPtr;
  if (!x || !y || !pkts || !out || !flags || bytes == 0 || (bytes % 16) != 0 || nblocks <= 0 || nblocks > kFlagSlots) return 4;
  if (nblocks % 2) nblocks += 1;
  const uint64_t nunits = bytes / 16;
#define SRV(U, SP, LP)                                                                                        \
  hipLaunchKernelGGL((selfReduceLL16Kernel<kF16, kSum, U, SP, LP>), dim3(nblocks), dim3(256), 0, s,           \
                     (const uint8_t*)x, (const uint8_t*)y, (uint8_t*)pkts, (uint8_t*)out, nunits, flags, budgetTicks, err)
  switch (variant) {
    case 0: SRV(4, kAgent, kSystem); break;
    case 1: SRV(2, kAgent, kSystem); break;
    case 2: SRV(8, kAgent, kSystem); break;
    case 3: SRV(4, kNonTemporal, kSystem); break;
    case 4: SRV(4, kPlain, kSystem); break;
    case 5: SRV(4, kAgent, kAgent); break;
    case 6: SRV(4, kSystem, kSystem); break;
    case 7: SRV(4, kNonTemporal, kAgent); break;
    case 8: SRV(8, kNonTemporal, kAgent); break;
    case 9: SRV(2, kNonTemporal, kAgent); break;
#define SRVPM(U, SP, LP)                                                                                      \
  hipLaunchKernelGGL((selfReduceLL16PmKernel<kF16, kSum, U, SP, LP>), dim3(nblocks), dim3(256), 0, s,         \
                     (const uint8_t*)x, (const uint8_t*)y, (uint8_t*)pkts, (uint8_t*)out, bytes / 8, flags, budgetTicks, err)
    case 10: SRVPM(8, kAgent, kSystem); break;
    case 11: SRVPM(4, kAgent, kSystem); break;
    case 12: SRVPM(16, kAgent, kSystem); break;
    case 13: SRVPM(8, kSystem, kSystem); break;
    case 14: SRVPM(8, kNonTemporal, kSystem); break;
    case 15: SRVPM(8, kAgent, kAgent); break;
#undef SRVPM
#define SRVLDS(U)                                                                                             \
  hipLaunchKernelGGL((selfReduceLL16LdsKernel<kF16, kSum, U>), dim3(nblocks), dim3(256), 0, s, (const uint8_t*)x, \
                     (const uint8_t*)y, (uint8_t*)pkts, (uint8_t*)out, (uint64_t)bytes, flags, budgetTicks, err)
    case 16: SRVLDS(4); break;
    case 17: SRVLDS(8); break;
    case 18: SRVLDS(2); break;
    case 19: SRVLDS(1); break;
#undef SRVLDS
    default: return 4;
  }
#undef SRV
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

extern "C" int mscclppAmdCopy(const void* src, void* dst, size_t bytes, int nblocks, void* streamPtr) {
  if (!src || !dst || bytes == 0 || (bytes % 16) != 0) return 4;
  if (nblocks <= 0) nblocks = 2048;
  hipLaunchKernelGGL((copyKernel<4>), dim3(nblocks), dim3(256), 0, (hipStream_t)streamPtr, (const uint8_t*)src,
                     (uint8_t*)dst, (uint64_t)(bytes / 16));
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

extern "C" int mscclppAmdSelfReduceLL16(const void* x, const void* y, void* pkts, void* out, size_t bytes, int dtype,
                                        int op, uint32_t* flags, int nblocks, uint64_t budgetTicks, uint32_t* err,
                                        void* streamPtr) {
  hipStream_t stream = (hipStream_t)streamPtr;
  if (!x || !y || !pkts || !out || !flags || bytes == 0 || (bytes % 16) != 0) return 4;
  if (nblocks <= 0) {
    // one 8 KiB payload tile per workgroup and round; 1024 workgroups = 4 per CU (8 KiB LDS each),
    // all resident, so every partner pair is co-resident
    const uint64_t tiles = (bytes + 8191) / 8192;
    nblocks = (int)(tiles < 1024 ? tiles : 1024);
  }
  if (nblocks % 2) nblocks += 1;
  if (nblocks > 1024) return 4;
  MSCCLPP_AMD_DISPATCH_ALL(dtype, op, launchSelfReduce, x, y, pkts, out, (uint64_t)bytes, flags, nblocks, budgetTicks, err, stream);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
