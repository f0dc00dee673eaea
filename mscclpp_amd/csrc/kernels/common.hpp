// Shared pieces of the mscclpp_amd kernels (not part of the public device API).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "mscclpp_amd/device.hpp"
#include "mscclpp_amd/mscclpp_amd.h"
#include "mscclpp_amd/packet_device.hpp"
#include "mscclpp_amd/reduce_device.hpp"

namespace mscclpp_amd {

// Flag slots shared by every packet kernel of a communicator (the reference keeps 128, initialised
// to 1: src/core/algorithm.cc:251-268).  A launch of G blocks uses slots [0, G); block 0 keeps the
// unused slots [G, kFlagSlots) equal so that a later launch with a larger grid reads the same flag
// in every block (allreduce_packet.cu:134-140).
constexpr int kFlagSlots = MSCCLPP_AMD_FLAG_SLOTS;
constexpr int kMaxRanks = MSCCLPP_AMD_MAX_RANKS;
constexpr int kMaxChannels = MSCCLPP_AMD_MAX_CHANNELS;

// Every workgroup of a collective kernel spins on workgroups of other ranks (and, with in-process
// ranks, of the same launch), so the whole grid must be resident at once.  Host side: true when
// `blocks` workgroups of `kernel` at `threads` lanes fit on the current device together.
// The answer is cached per kernel instantiation, device and block size (launches stay cheap).
template <typename Kernel>
inline bool grid_coresident(Kernel kernel, int threads, long blocks) {
  static thread_local Kernel cKernel = nullptr;
  static thread_local int cDev = -1, cThreads = -1;
  static thread_local long cCap = 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  if (kernel != cKernel || dev != cDev || threads != cThreads) {
    int cus = 0, per = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return false;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, threads, 0) != hipSuccess) {
      fprintf(stderr, "[mscclpp_amd WARN] occupancy query failed: %s\n", hipGetErrorString(hipGetLastError()));
      return false;
    }
    cKernel = kernel;
    cDev = dev;
    cThreads = threads;
    cCap = (long)per * cus;
  }
  if (cCap < blocks)
    fprintf(stderr, "[mscclpp_amd WARN] %ld workgroups of %d lanes cannot be co-resident (device %d holds %ld)\n",
            blocks, threads, dev, cCap);
  return cCap >= blocks;
}

// (`flags` is 16-byte aligned: block 0 refreshes the slots above the grid with 16-byte stores, a
// quarter of the instructions of word stores: 4 per lane instead of 16 for a 16-workgroup grid)
__device__ __forceinline__ void bump_flags(uint32_t* flags, uint32_t flag) {
  __syncthreads();
  const uint32_t v = flag + 1;
  if (threadIdx.x == 0) flags[blockIdx.x] = v;
  if (blockIdx.x == 0) {
    const uint32_t g = gridDim.x, a = (g + 3u) & ~3u;  // first slot of a whole 16-byte group above the grid
    if (threadIdx.x < a - g && g + threadIdx.x < (uint32_t)kFlagSlots) flags[g + threadIdx.x] = v;
    const auto r = make_rsrc(flags);
    for (uint32_t i = a / 4 + threadIdx.x; i < (uint32_t)kFlagSlots / 4; i += blockDim.x)
      store16<kPlain>(r, i * 16u, u32x4{v, v, v, v});
  }
}

__device__ __forceinline__ uint32_t wave_uniform(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// Phase trace (the role of the reference's NPKit events, allreduce_packet.cu:20-49, npkit.hpp):
// with a trace buffer set through mscclppAmdTraceSet, lane 0 of every workgroup stamps the wall
// clock (s_memrealtime, 10 ns) at the kernel's phase boundaries into
// trace[(view * kTraceBlocks + block) * kTraceEvents + event], view = the in-process rank index
// (0 with one rank per process).  Without one the stamps cost one scalar branch each.  The stamp
// is lane 0's own view of the phase (the other lanes of the workgroup may still be in it).  Only
// workgroups below kTraceBlocks (and views below kMaxRanks) stamp, so the buffer bound holds.
constexpr int kTraceEvents = 8;
constexpr int kTraceBlocks = kMaxChannels;
__device__ __forceinline__ void trace_stamp(uint64_t* trace, int event) {
  if (trace && threadIdx.x == 0 && blockIdx.x < (uint32_t)kTraceBlocks && blockIdx.y < (uint32_t)kMaxRanks) {
    const uint64_t t = wall_ticks();
    const uint32_t slot = ((uint32_t)blockIdx.y * kTraceBlocks + blockIdx.x) * kTraceEvents + (uint32_t)event;
    store8<kPlain>(make_rsrc(trace), slot * 8u, u32x2{(uint32_t)t, (uint32_t)(t >> 32)});
  }
}

// Kernel argument carrying NV rank views (NV = 1: one rank per process; NV = n: in-process ranks).
template <int NV>
struct Views {
  mscclppAmdRankView v[NV];
};

// Payload tail helpers: a 16-byte unit of which only `valid` (< 16) bytes lie inside the buffer.
__device__ __forceinline__ u32x4 load_tail(const uint8_t* p, uint32_t valid) {
  uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if ((uint32_t)i < valid) w[i / 4] |= (uint32_t)p[i] << ((i % 4) * 8);
  return u32x4{w[0], w[1], w[2], w[3]};
}
__device__ __forceinline__ void store_tail(uint8_t* p, u32x4 v, uint32_t valid) {
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if ((uint32_t)i < valid) p[i] = (uint8_t)(w[i / 4] >> ((i % 4) * 8));
}

// Load the 16-byte payload unit at byte `off` of buffer `base` (rsrc `r` over the same base) whose
// first `valid` bytes are in range.
template <int Policy>
__device__ __forceinline__ u32x4 load_payload(__amdgpu_buffer_rsrc_t r, const uint8_t* base, uint64_t off,
                                              uint32_t valid) {
  if (valid >= 16) return load16<Policy>(r, (uint32_t)off);
  return load_tail(base + off, valid);
}
template <int Policy>
__device__ __forceinline__ void store_payload(__amdgpu_buffer_rsrc_t r, uint8_t* base, uint64_t off, u32x4 v,
                                              uint32_t valid) {
  if (valid >= 16)
    store16<Policy>(r, (uint32_t)off, v);
  else
    store_tail(base + off, v, valid);
}

__device__ __forceinline__ uint32_t clamp_valid(uint64_t total, uint64_t off, uint32_t cap) {
  if (off >= total) return 0;
  uint64_t rem = total - off;
  return rem < cap ? (uint32_t)rem : cap;
}

}  // namespace mscclpp_amd

// The trace buffer the next launches stamp into (null: off); set by mscclppAmdTraceSet.
extern uint64_t* g_mscclppAmdTrace;
