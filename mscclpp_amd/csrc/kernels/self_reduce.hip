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
// grid at or below 2 workgroups per CU (256 CUs).  Every spin is time-bounded.
//
// Algorithmic HBM bytes per launch: 7*S (Y read S, P written 2S, P read 2S, X read S, O written S).
#include "common.hpp"

namespace mscclpp_amd {

template <int DT, int OP, int U, int PKT_POLICY>
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

  for (uint64_t base = 0; base < ntiles; base += G) {
    // ---- pack my tile
    const uint64_t t = base + b;
    if (t < ntiles) {
      const uint64_t u0 = t * kTileUnits;
      auto ry = make_rsrc(y + u0 * 16);
      auto rp = make_rsrc(pkts + u0 * 32);
      u32x4 w[U];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const uint64_t u = u0 + k * kThreads + tid;
        if (u < nunits) w[k] = load16<kNonTemporal>(ry, (uint32_t)((k * kThreads + tid) * 16));
      }
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const uint64_t u = u0 + k * kThreads + tid;
        if (u < nunits) ll16_put_unit<PKT_POLICY>(rp, (uint32_t)((k * kThreads + tid) * 32), w[k], flag);
      }
    }
    // ---- consume my partner's tile
    const uint64_t tp = base + partner;
    if (partner < G && tp < ntiles) {
      const uint64_t u0 = tp * kTileUnits;
      auto rx = make_rsrc(x + u0 * 16);
      auto ro = make_rsrc(out + u0 * 16);
      auto rp = make_rsrc(pkts + u0 * 32);
      u32x4 v[U], a[U];
      bool ok = true;
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const uint64_t u = u0 + k * kThreads + tid;
        if (u < nunits) {
          a[k] = load16<kNonTemporal>(rx, (uint32_t)((k * kThreads + tid) * 16));
          ok &= ll16_try_unit(rp, (uint32_t)((k * kThreads + tid) * 32), flag, v[k]);
        }
      }
      if (!ok) {
#pragma unroll
        for (int k = 0; k < U; ++k) {
          const uint64_t u = u0 + k * kThreads + tid;
          if (u < nunits) v[k] = ll16_get_unit(rp, (uint32_t)((k * kThreads + tid) * 32), flag, budget, err);
        }
      }
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const uint64_t u = u0 + k * kThreads + tid;
        if (u < nunits) store16<kNonTemporal>(ro, (uint32_t)((k * kThreads + tid) * 16), reduce4<DT, OP>(a[k], v[k]));
      }
    }
  }
  bump_flags(flags, flag);
}

template <int DT, int OP>
static void launchSelfReduce(const void* x, const void* y, void* pkts, void* out, uint64_t nunits, uint32_t* flags,
                             int nblocks, uint64_t budget, uint32_t* err, hipStream_t stream) {
  hipLaunchKernelGGL((selfReduceLL16Kernel<DT, OP, 4, kAgent>), dim3(nblocks), dim3(256), 0, stream,
                     (const uint8_t*)x, (const uint8_t*)y, (uint8_t*)pkts, (uint8_t*)out, nunits, flags, budget, err);
}

}  // namespace mscclpp_amd

using namespace mscclpp_amd;

extern "C" int mscclppAmdSelfReduceLL16(const void* x, const void* y, void* pkts, void* out, size_t bytes, int dtype,
                                        int op, uint32_t* flags, int nblocks, uint64_t budgetTicks, uint32_t* err,
                                        void* streamPtr) {
  hipStream_t stream = (hipStream_t)streamPtr;
  if (!x || !y || !pkts || !out || !flags || bytes == 0 || (bytes % 16) != 0) return 4;
  if (nblocks <= 0) {
    // one 16 KiB payload tile per workgroup and round; at most 2 workgroups per CU so every pair
    // is resident (see the header comment)
    const uint64_t tiles = (bytes + 16383) / 16384;
    nblocks = (int)(tiles < 512 ? tiles : 512);
  }
  if (nblocks % 2) nblocks += 1;
  if (nblocks > 512) return 4;
  const uint64_t nunits = bytes / 16;
  MSCCLPP_AMD_DISPATCH(dtype, op, launchSelfReduce, x, y, pkts, out, nunits, flags, nblocks, budgetTicks, err, stream);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
