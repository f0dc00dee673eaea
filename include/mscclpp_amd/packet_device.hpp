// LL (low-latency) packets for gfx950.
//
// Memory images are identical to the reference (include/mscclpp/packet_device.hpp:19-159):
//   LL16 packet i = u32[4] {data1 = P[2i], flag1 = f, data2 = P[2i+1], flag2 = f}  (8 payload bytes)
//   LL8  packet i = u32[2] {data = P[i], flag = f}                                 (4 payload bytes)
// A reader accepts a packet only when every flag word equals the expected flag.
//
// What differs is how the bytes move.  The reference writes an LL16 packet as two 8-byte
// nontemporal stores and polls with two 8-byte relaxed atomic loads (packet_device.hpp:45-48,
// :74-80).  Here one lane moves a whole packet with one 16-byte buffer access carrying the cache
// policy of the hop (sc0 sc1 = system scope for peer GPUs, sc1 for another XCD of the same GPU).
// Each naturally aligned 8-byte half carries its own flag, so a 16-byte access torn into halves is
// still read correctly; the hot loops additionally move two packets (16 payload bytes) per lane so
// that the payload side is a full dwordx4 as well.
#pragma once

#include "device.hpp"

namespace mscclpp_amd {

union alignas(16) LL16Packet {
  struct {
    uint32_t data1;
    uint32_t flag1;
    uint32_t data2;
    uint32_t flag2;
  };
  u32x4 raw;

  using Payload = uint2;  // packet_device.hpp:27

  LL16Packet() = default;
  __device__ __forceinline__ LL16Packet(uint2 val, uint32_t flag) : raw(make(val.x, val.y, flag)) {}

  __device__ __forceinline__ static u32x4 make(uint32_t v1, uint32_t v2, uint32_t flag) {
    u32x4 p;
    p.x = v1;
    p.y = flag;
    p.z = v2;
    p.w = flag;
    return p;
  }
  __device__ __forceinline__ static bool ready(u32x4 p, uint32_t flag) { return p.y == flag && p.w == flag; }

  // Single-packet write through a raw pointer (system scope, write-through: one 16-byte store whose
  // two 8-byte halves each carry the flag).  Hot loops use the buffer-resource forms below.
  __device__ __forceinline__ void write(uint32_t v1, uint32_t v2, uint32_t flag) {
    u32x4 p = make(v1, v2, flag);
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(&raw), "v"(p) : "memory");
  }
  __device__ __forceinline__ void write(uint64_t val, uint32_t flag) { write((uint32_t)val, (uint32_t)(val >> 32), flag); }
  __device__ __forceinline__ void write(uint2 val, uint32_t flag) { write(val.x, val.y, flag); }

  // One poll: two relaxed system-scope 8-byte loads.  Returns true when both flags match.
  __device__ __forceinline__ bool readOnce(uint32_t flag, uint32_t& v1, uint32_t& v2) const {
    const uint64_t* q = reinterpret_cast<const uint64_t*>(this);
    uint64_t lo = ld_relaxed_sys(q), hi = ld_relaxed_sys(q + 1);
    v1 = (uint32_t)lo;
    v2 = (uint32_t)hi;
    return (uint32_t)(lo >> 32) == flag && (uint32_t)(hi >> 32) == flag;
  }
  // The reference's helper of read() (packet_device.hpp:66-82): true while the flags do NOT match.
  __device__ __forceinline__ bool readOnce(uint32_t flag, uint2& data) const {
    uint32_t v1, v2;
    const bool ok = readOnce(flag, v1, v2);
    data.x = v1;
    data.y = v2;
    return !ok;
  }
  // Spin until both flags match; on timeout record kErrPacketTimeout with the flag, `where` (the
  // packet's byte offset in its region) and the flag word seen, and return zeros.
  __device__ __forceinline__ bool read(uint32_t flag, uint32_t& v1, uint32_t& v2, uint64_t budget, uint32_t* err,
                                       uint64_t where = 0) const {
    SpinGuard g(budget);
    while (!readOnce(flag, v1, v2)) {
      if (g.expired()) {
        const uint64_t* q = reinterpret_cast<const uint64_t*>(this);
        const uint32_t f1 = (uint32_t)(ld_relaxed_sys(q) >> 32), f2 = (uint32_t)(ld_relaxed_sys(q + 1) >> 32);
        report_packet_timeout(err, flag, where, f1 != flag ? f1 : f2);
        v1 = v2 = 0;
        return false;
      }
    }
    return true;
  }
  // The reference's read (packet_device.hpp:88-92): the payload once both flags match.  Bounded by
  // kDefaultSpinTicks of wall clock (maxSpinCount: see device.hpp); after a timeout it returns the
  // last payload seen.
  __device__ __forceinline__ uint2 read(uint32_t flag, int64_t maxSpinCount = 100000000) const {
    (void)maxSpinCount;
    uint32_t v1, v2;
    SpinGuard g(kDefaultSpinTicks);
    while (!readOnce(flag, v1, v2) && !g.expired()) {
    }
    uint2 d;
    d.x = v1;
    d.y = v2;
    return d;
  }
  __device__ __forceinline__ void clear() { raw = u32x4{0, 0, 0, 0}; }
};

union alignas(8) LL8Packet {
  struct {
    uint32_t data;
    uint32_t flag;
  };
  uint64_t raw;

  using Payload = uint32_t;  // packet_device.hpp:108

  LL8Packet() = default;
  __device__ __forceinline__ LL8Packet(uint32_t val, uint32_t f) : raw(make(val, f)) {}

  __device__ __forceinline__ static uint64_t make(uint32_t v, uint32_t flag) { return ((uint64_t)flag << 32) | v; }
  // One relaxed system-scope 8-byte store (packet_device.hpp:118-126).
  __device__ __forceinline__ void write(uint32_t v, uint32_t flag) {
    __hip_atomic_store(&raw, make(v, flag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // The reference's helper of read() (packet_device.hpp:132-144): true while the flag does NOT match.
  __device__ __forceinline__ bool readOnce(uint32_t flag, uint32_t& data) const {
    uint64_t x = ld_relaxed_sys(&raw);
    data = (uint32_t)x;
    return (uint32_t)(x >> 32) != flag;
  }
  __device__ __forceinline__ bool read(uint32_t flag, uint32_t& v, uint64_t budget, uint32_t* err,
                                       uint64_t where = 0) const {
    SpinGuard g(budget);
    while (readOnce(flag, v)) {
      if (g.expired()) {
        report_packet_timeout(err, flag, where, (uint32_t)(ld_relaxed_sys(&raw) >> 32));
        v = 0;
        return false;
      }
    }
    return true;
  }
  // The reference's read (packet_device.hpp:150-154), bounded by kDefaultSpinTicks of wall clock.
  __device__ __forceinline__ uint32_t read(uint32_t flag, int64_t maxSpinCount = 1000000) const {
    (void)maxSpinCount;
    uint32_t v;
    SpinGuard g(kDefaultSpinTicks);
    while (readOnce(flag, v) && !g.expired()) {
    }
    return v;
  }
  __device__ __forceinline__ void clear() { raw = 0; }
};

using LLPacket = LL16Packet;  // packet_device.hpp:161

// ---------------------------------------------------------------------------------------------
// Packet streams: the hot-loop forms.  A "unit" is 16 payload bytes = 2 LL16 packets (32 B) or
// 4 LL8 packets (32 B).  Unit u of a payload region maps to packet bytes [32u, 32u + 32).
// ---------------------------------------------------------------------------------------------

// Pack one unit: payload words w -> two LL16 packets at packet byte offset `pbyte`.
template <int Policy>
__device__ __forceinline__ void ll16_put_unit(__amdgpu_buffer_rsrc_t pkts, uint32_t pbyte, u32x4 w, uint32_t flag) {
  store16<Policy>(pkts, pbyte, LL16Packet::make(w.x, w.y, flag));
  store16<Policy>(pkts, pbyte + 16, LL16Packet::make(w.z, w.w, flag));
}

// Poll one unit once.  Returns true and fills w when both packets carry `flag`.
template <int LoadPolicy = kSystem>
__device__ __forceinline__ bool ll16_try_unit(__amdgpu_buffer_rsrc_t pkts, uint32_t pbyte, uint32_t flag, u32x4& w) {
  u32x4 a = load16<LoadPolicy>(pkts, pbyte);
  u32x4 b = load16<LoadPolicy>(pkts, pbyte + 16);
  w.x = a.x;
  w.y = a.z;
  w.z = b.x;
  w.w = b.z;
  return LL16Packet::ready(a, flag) && LL16Packet::ready(b, flag);
}

// Timeout detail of a 32-byte unit (two LL16 or four LL8 packets; flag words 1 and 3 of each
// 16 bytes): the first flag word that differs from `flag`, re-read once.
template <int LoadPolicy>
__device__ __forceinline__ uint32_t unit_flag_seen(__amdgpu_buffer_rsrc_t pkts, uint32_t pbyte, uint32_t flag) {
  const u32x4 a = load16<LoadPolicy>(pkts, pbyte), b = load16<LoadPolicy>(pkts, pbyte + 16);
  return a.y != flag ? a.y : a.w != flag ? a.w : b.y != flag ? b.y : b.w;
}

template <int LoadPolicy = kSystem>
__device__ __forceinline__ u32x4 ll16_get_unit(__amdgpu_buffer_rsrc_t pkts, uint32_t pbyte, uint32_t flag,
                                               uint64_t budget, uint32_t* err) {
  u32x4 w;
  if (ll16_try_unit<LoadPolicy>(pkts, pbyte, flag, w)) return w;
  SpinGuard g(budget);
  while (!ll16_try_unit<LoadPolicy>(pkts, pbyte, flag, w)) {
    if (g.expired()) {
      report_packet_timeout(err, flag, pbyte, unit_flag_seen<LoadPolicy>(pkts, pbyte, flag));
      return u32x4{0, 0, 0, 0};
    }
  }
  return w;
}

template <int Policy>
__device__ __forceinline__ void ll8_put_unit(__amdgpu_buffer_rsrc_t pkts, uint32_t pbyte, u32x4 w, uint32_t flag) {
  u32x4 a, b;
  a.x = w.x;
  a.y = flag;
  a.z = w.y;
  a.w = flag;
  b.x = w.z;
  b.y = flag;
  b.z = w.w;
  b.w = flag;
  store16<Policy>(pkts, pbyte, a);
  store16<Policy>(pkts, pbyte + 16, b);
}

__device__ __forceinline__ bool ll8_try_unit(__amdgpu_buffer_rsrc_t pkts, uint32_t pbyte, uint32_t flag, u32x4& w) {
  u32x4 a = load16<kSystem>(pkts, pbyte);
  u32x4 b = load16<kSystem>(pkts, pbyte + 16);
  w.x = a.x;
  w.y = a.z;
  w.z = b.x;
  w.w = b.z;
  return a.y == flag && a.w == flag && b.y == flag && b.w == flag;
}

__device__ __forceinline__ u32x4 ll8_get_unit(__amdgpu_buffer_rsrc_t pkts, uint32_t pbyte, uint32_t flag,
                                              uint64_t budget, uint32_t* err) {
  u32x4 w;
  if (ll8_try_unit(pkts, pbyte, flag, w)) return w;
  SpinGuard g(budget);
  while (!ll8_try_unit(pkts, pbyte, flag, w)) {
    if (g.expired()) {
      report_packet_timeout(err, flag, pbyte, unit_flag_seen<kSystem>(pkts, pbyte, flag));
      return u32x4{0, 0, 0, 0};
    }
  }
  return w;
}

// Threaded helpers with an explicit spin budget and error word (the budget/error-word overloads of
// copyToPackets / copyFromPackets, copy_device.hpp:156-232; the reference-spelled templates are in
// copy_device.hpp): thread `tid` of `nthreads` handles packets tid, tid + nthreads, ...
__device__ __forceinline__ void copyToPacketsLL16(void* dst, const void* src, uint64_t bytes, uint32_t tid,
                                                  uint32_t nthreads, uint32_t flag) {
  const uint32_t* s = reinterpret_cast<const uint32_t*>(src);
  LL16Packet* d = reinterpret_cast<LL16Packet*>(dst);
  for (uint64_t i = tid; i < bytes / 8; i += nthreads) d[i].write(s[2 * i], s[2 * i + 1], flag);
}
__device__ __forceinline__ void copyFromPacketsLL16(void* dst, const void* src, uint64_t bytes, uint32_t tid,
                                                    uint32_t nthreads, uint32_t flag, uint64_t budget, uint32_t* err) {
  const LL16Packet* s = reinterpret_cast<const LL16Packet*>(src);
  uint32_t* d = reinterpret_cast<uint32_t*>(dst);
  for (uint64_t i = tid; i < bytes / 8; i += nthreads) {
    uint32_t v1, v2;
    s[i].read(flag, v1, v2, budget, err, i * 16);
    d[2 * i] = v1;
    d[2 * i + 1] = v2;
  }
}
__device__ __forceinline__ void copyToPacketsLL8(void* dst, const void* src, uint64_t bytes, uint32_t tid,
                                                 uint32_t nthreads, uint32_t flag) {
  const uint32_t* s = reinterpret_cast<const uint32_t*>(src);
  LL8Packet* d = reinterpret_cast<LL8Packet*>(dst);
  for (uint64_t i = tid; i < bytes / 4; i += nthreads) d[i].write(s[i], flag);
}
__device__ __forceinline__ void copyFromPacketsLL8(void* dst, const void* src, uint64_t bytes, uint32_t tid,
                                                   uint32_t nthreads, uint32_t flag, uint64_t budget, uint32_t* err) {
  const LL8Packet* s = reinterpret_cast<const LL8Packet*>(src);
  uint32_t* d = reinterpret_cast<uint32_t*>(dst);
  for (uint64_t i = tid; i < bytes / 4; i += nthreads) {
    uint32_t v;
    s[i].read(flag, v, budget, err, i * 8);
    d[i] = v;
  }
}

}  // namespace mscclpp_amd
