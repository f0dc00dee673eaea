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
// and is handed out again, its requested bytes zeroed, for a later request of its size class on the
// same device -- after one device synchronize at that reuse (a free never synchronizes: kernels
// queued before it may still use the block, so it waits in a pending list until then).
//
// Size classes: powers of two from 64 KiB up to 64 MiB; above that, multiples of 2 MiB (a 129 MiB
// scratch holds 130 MiB, not 256).  A large request is served best-fit by a free block of at most
// 5/4 of its class.  The held bytes are bounded by the peak of what was live at once, per class
// (INTEGRATION.md §5); mscclppAmdUncachedPoolStats reports them.
// MSCCLPP_AMD_UC_POOL=0 restores hipFree (diagnosis only).
#include "comm_internal.hpp"

#include <unordered_map>

namespace mscclpp_amd {
namespace host {
namespace {

struct Block {
  int device;
  size_t cls;
};

struct UncachedPool {
  std::mutex mu;
  std::map<std::pair<int, size_t>, std::vector<void*>> freeBlocks;  // (device, class bytes) -> blocks
  // freed by their owner, but kernels queued before the free may still use them: they join the free
  // lists at the next device synchronize, which only an allocation that could reuse them pays
  std::map<std::pair<int, size_t>, std::vector<void*>> pending;
  std::unordered_map<void*, Block> live;                            // block -> owner device, class
  std::map<int, hipStream_t> zeroStreams;  // per device: the stream the zero fill runs on
  size_t held = 0;                         // bytes allocated from HIP and never freed
  size_t leaked = 0;                       // bytes dropped because their device could not synchronize
  bool enabled = [] {
    const char* e = std::getenv("MSCCLPP_AMD_UC_POOL");
    return !(e && std::string(e) == "0");
  }();
};

UncachedPool& pool() {
  static UncachedPool* p = new UncachedPool();  // never destroyed: blocks outlive static teardown
  return *p;
}

constexpr size_t kPow2Max = (size_t)64 << 20;
constexpr size_t kLargeStep = (size_t)2 << 20;

size_t classOf(size_t bytes) {
  if (bytes > kPow2Max) return (bytes + kLargeStep - 1) / kLargeStep * kLargeStep;
  size_t c = (size_t)64 << 10;
  while (c < bytes) c <<= 1;
  return c;
}

// A free block of `cls` on `dev` (caller holds the lock): the exact class, or for a large class the
// smallest free one up to 5/4 of it.
void* takeFree(UncachedPool& P, int dev, size_t cls, size_t* got) {
  auto it = P.freeBlocks.lower_bound({dev, cls});
  const size_t limit = cls > kPow2Max ? cls + cls / 4 : cls;
  for (; it != P.freeBlocks.end() && it->first.first == dev && it->first.second <= limit; ++it) {
    if (it->second.empty()) continue;
    void* p = it->second.back();
    it->second.pop_back();
    *got = it->first.second;
    return p;
  }
  return nullptr;
}

// Is a pending block of `dev` able to serve `cls` (caller holds the lock)?
bool pendingFits(UncachedPool& P, int dev, size_t cls) {
  auto it = P.pending.lower_bound({dev, cls});
  const size_t limit = cls > kPow2Max ? cls + cls / 4 : cls;
  for (; it != P.pending.end() && it->first.first == dev && it->first.second <= limit; ++it)
    if (!it->second.empty()) return true;
  return false;
}

// Move the pending blocks of `dev` to the free lists once the device has drained (the current
// device is `dev`); blocks of a device that cannot synchronize are leaked.  Only the blocks pending
// BEFORE the synchronize are moved: they are taken out under the lock first, then the device is
// synchronized, then they join the free lists.  A block another thread releases in between (its
// kernels possibly queued after the synchronize returned) stays pending until the next drain.
void drainPending(UncachedPool& P, int dev) {
  std::vector<std::pair<size_t, void*>> snapshot;
  {
    std::lock_guard<std::mutex> lk(P.mu);
    for (auto it = P.pending.lower_bound({dev, 0}); it != P.pending.end() && it->first.first == dev; ++it) {
      for (void* b : it->second) snapshot.emplace_back(it->first.second, b);
      it->second.clear();
    }
  }
  const hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) (void)hipGetLastError();
  std::lock_guard<std::mutex> lk(P.mu);
  for (const auto& sb : snapshot) {
    if (e == hipSuccess) P.freeBlocks[{dev, sb.first}].push_back(sb.second);
    else P.leaked += sb.first;
  }
}

// Zero the first `bytes` of a block of `dev`.
void zeroFill(UncachedPool& P, int dev, void* p, size_t bytes) {
  // The fill runs on a stream created for it and destroyed after it (default): never the null
  // stream (a legacy-stream memset would join, or break, another thread's graph capture), and no
  // stream left behind -- a persistent extra stream in the process made every PortChannel put
  // 1.4-1.7x slower (round 4: 108 -> 183 us putWithSignal at 1 MiB; tools/portchannel_ab.py,
  // profiles/r5_portchannel_ab.json).  MSCCLPP_AMD_POOL_ZERO (diagnosis): "legacy" = the null-stream
  // hipMemset of round 3, "stream" = the persistent per-device stream of round 4.
  static const int how = [] {
    const char* e = std::getenv("MSCCLPP_AMD_POOL_ZERO");
    const std::string v = e ? e : "";
    return v == "legacy" ? 1 : v == "stream" ? 0 : 2;
  }();
  if (how == 1) {
    HIPCHECK(hipMemset(p, 0, bytes));
    return;
  }
  if (how == 2) {
    hipStream_t t = nullptr;
    HIPCHECK(hipStreamCreateWithFlags(&t, hipStreamNonBlocking));
    const hipError_t e1 = hipMemsetAsync(p, 0, bytes, t);
    const hipError_t e2 = e1 == hipSuccess ? hipStreamSynchronize(t) : e1;
    (void)hipStreamDestroy(t);
    HIPCHECK(e2);
    return;
  }
  hipStream_t s = nullptr;
  {
    std::lock_guard<std::mutex> lk(P.mu);
    auto it = P.zeroStreams.find(dev);
    if (it != P.zeroStreams.end()) s = it->second;
  }
  if (!s) {
    HIPCHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::lock_guard<std::mutex> lk(P.mu);
    auto ins = P.zeroStreams.emplace(dev, s);
    if (!ins.second) {  // another thread created one first
      (void)hipStreamDestroy(s);
      s = ins.first->second;
    }
  }
  HIPCHECK(hipMemsetAsync(p, 0, bytes, s));
  HIPCHECK(hipStreamSynchronize(s));
}

}  // namespace

void* allocUncached(size_t bytes) {
  UncachedPool& P = pool();
  int dev = 0;
  HIPCHECK(hipGetDevice(&dev));
  void* p = nullptr;
  size_t cls = bytes;
  {
    std::lock_guard<std::mutex> lk(P.mu);
    if (P.enabled) {
      cls = classOf(bytes);
      size_t got = 0;
      p = takeFree(P, dev, cls, &got);
      if (p) {
        cls = got;
        P.live[p] = Block{dev, cls};
      }
    }
  }
  if (!p && P.enabled) {
    bool reuse = false;
    {
      std::lock_guard<std::mutex> lk(P.mu);
      reuse = pendingFits(P, dev, cls);
    }
    if (reuse) {  // a freed block fits: wait for the device once, then take it
      drainPending(P, dev);
      std::lock_guard<std::mutex> lk(P.mu);
      size_t got = 0;
      p = takeFree(P, dev, cls, &got);
      if (p) {
        cls = got;
        P.live[p] = Block{dev, cls};
      }
    }
  }
  if (!p) {
    HIPCHECK(hipExtMallocWithFlags(&p, cls, hipDeviceMallocUncached));
    std::lock_guard<std::mutex> lk(P.mu);
    if (P.enabled) {
      P.live[p] = Block{dev, cls};
      P.held += cls;
    }
  }
  try {
    zeroFill(P, dev, p, bytes);
  } catch (...) {  // the caller never receives the block: it must not stay live (counted, never reused)
    std::lock_guard<std::mutex> lk(P.mu);
    if (P.live.erase(p)) P.pending[{dev, cls}].push_back(p);
    else (void)hipFree(p);
    throw;
  }
  return p;
}

void memsetSync(void* p, int value, size_t bytes) {
  if (!p || bytes == 0) return;
  hipStream_t s = nullptr;
  HIPCHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipError_t e = hipMemsetAsync(p, value, bytes, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipStreamDestroy(s);
  HIPCHECK(e);
}

bool releaseUncached(void* p, hipError_t* syncError) noexcept {
  if (syncError) *syncError = hipSuccess;
  if (!p) return true;
  UncachedPool& P = pool();
  // No synchronize here: the block waits in `pending` -- kernels queued before
  // this free may still use it -- until an allocation that could reuse it drains the device once
  // (as hipFree would have, but only when reuse is possible, never on the free path).
  std::lock_guard<std::mutex> lk(P.mu);
  auto it = P.live.find(p);
  if (it == P.live.end()) return false;  // not a pooled block
  P.pending[{it->second.device, it->second.cls}].push_back(p);
  P.live.erase(it);
  return true;
}

void freeDevice(void* p) noexcept {
  if (!p) return;
  if (!releaseUncached(p, nullptr)) (void)hipFree(p);
}

bool isPooledUncached(const void* base) {
  UncachedPool& P = pool();
  std::lock_guard<std::mutex> lk(P.mu);
  return P.live.count(const_cast<void*>(base)) != 0;
}

void uncachedPoolStats(size_t* held, size_t* inUse, size_t* freeBytes) {
  UncachedPool& P = pool();
  std::lock_guard<std::mutex> lk(P.mu);
  size_t used = 0, fr = 0;
  for (const auto& e : P.live) used += e.second.cls;
  for (const auto& e : P.freeBlocks) fr += e.first.second * e.second.size();
  for (const auto& e : P.pending) fr += e.first.second * e.second.size();
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
