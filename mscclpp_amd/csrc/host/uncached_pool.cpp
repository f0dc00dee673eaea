// Process-lifetime pool of uncached device memory (hipDeviceMallocUncached, the reference's
// GpuBuffer on AMD, gpu_utils.cc:139-147): every scratch, token and packet buffer of this library.
//
// Why a pool: in a long-lived process, a coarse-grained allocation (PyTorch's
// caching allocator) placed at the virtual range of a freed uncached allocation stopped receiving
// kernel stores as the copy engine sees them -- every XCD read the stored values back, a
// device-to-host copy read the bytes the buffer held before the kernel -- so a correct AllReduce
// result came back wrong through .cpu() (k5 in the full `-m gpu` session, 6 of 6 sessions; the
// buffer sat exactly where 1-2 MiB uncached buffers had been allocated and freed).  Uncached memory
// is therefore never returned to HIP while the process runs: a freed block goes to a free list
// (after a device synchronize, as hipFree does) and is handed out again, zeroed, for a later request
// of its size class.  MSCCLPP_AMD_UC_POOL=0 restores hipFree (diagnosis only).
#include "comm_internal.hpp"

#include <unordered_map>

namespace mscclpp_amd {
namespace host {
namespace {

struct UncachedPool {
  std::mutex mu;
  std::multimap<size_t, void*> freeBlocks;   // class bytes -> block
  std::unordered_map<void*, size_t> live;    // block -> class bytes
  size_t held = 0;                           // bytes allocated from HIP and never freed
  bool enabled = [] {
    const char* e = std::getenv("MSCCLPP_AMD_UC_POOL");
    return !(e && std::string(e) == "0");
  }();
};

UncachedPool& pool() {
  static UncachedPool* p = new UncachedPool();  // never destroyed: blocks outlive static teardown
  return *p;
}

// Size classes: powers of two from 64 KiB, so a block serves requests down to half its size.
size_t classOf(size_t bytes) {
  size_t c = (size_t)64 << 10;
  while (c < bytes) c <<= 1;
  return c;
}

}  // namespace

void* allocUncached(size_t bytes) {
  UncachedPool& P = pool();
  void* p = nullptr;
  size_t cls = bytes;
  {
    std::lock_guard<std::mutex> lk(P.mu);
    if (P.enabled) {
      cls = classOf(bytes);
      auto it = P.freeBlocks.find(cls);
      if (it != P.freeBlocks.end()) {
        p = it->second;
        P.freeBlocks.erase(it);
        P.live[p] = cls;
      }
    }
  }
  if (!p) {
    HIPCHECK(hipExtMallocWithFlags(&p, cls, hipDeviceMallocUncached));
    std::lock_guard<std::mutex> lk(P.mu);
    if (P.enabled) {
      P.live[p] = cls;
      P.held += cls;
    }
  }
  HIPCHECK(hipMemset(p, 0, cls));
  return p;
}

bool releaseUncached(void* p) {
  if (!p) return true;
  UncachedPool& P = pool();
  {
    std::lock_guard<std::mutex> lk(P.mu);
    if (P.live.find(p) == P.live.end()) return false;  // not a pooled block
  }
  // as hipFree: no queued kernel may still use the block when it is handed out again
  HIPCHECK(hipDeviceSynchronize());
  std::lock_guard<std::mutex> lk(P.mu);
  auto it = P.live.find(p);
  if (it == P.live.end()) return true;
  P.freeBlocks.emplace(it->second, p);
  P.live.erase(it);
  return true;
}

void freeDevice(void* p) {
  if (!p) return;
  if (!releaseUncached(p)) (void)hipFree(p);
}

void uncachedPoolStats(size_t* held, size_t* inUse, size_t* freeBytes) {
  UncachedPool& P = pool();
  std::lock_guard<std::mutex> lk(P.mu);
  size_t used = 0, fr = 0;
  for (const auto& e : P.live) used += e.second;
  for (const auto& e : P.freeBlocks) fr += e.first;
  if (held) *held = P.held;
  if (inUse) *inUse = used;
  if (freeBytes) *freeBytes = fr;
}

}  // namespace host
}  // namespace mscclpp_amd

extern "C" int mscclppAmdUncachedPoolStats(size_t* held, size_t* inUse, size_t* freeBytes) {
  return mscclpp_amd::host::guarded([&] {
    mscclpp_amd::host::uncachedPoolStats(held, inUse, freeBytes);
    return (int)ncclSuccess;
  });
}
