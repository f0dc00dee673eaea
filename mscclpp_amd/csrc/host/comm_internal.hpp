// Internal host-runtime declarations shared by comm.cpp and proxy.cpp (not installed).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

#include "bootstrap.hpp"
#include "mscclpp_amd/algorithm.hpp"
#include "mscclpp_amd/mscclpp_amd.h"
#include "mscclpp_amd/nccl.h"

namespace mscclpp_amd {
int launchAllReduceLL(int algo, const mscclppAmdRankView* views, int nviews, int nranks, size_t bytes, int dtype,
                      int op, int nblocks, int nthreads, uint64_t budget, hipStream_t s);
int launchCollectiveBulk(int mode, int algo, const mscclppAmdRankView* views, int nviews, int nranks, size_t bytes,
                         int dtype, int op, int nblocks, int nthreads, uint64_t budget, hipStream_t s);
int launchAllReduceBulk(int algo, const mscclppAmdRankView* views, int nviews, int nranks, size_t bytes, int dtype,
                        int op, int nblocks, int nthreads, uint64_t budget, hipStream_t s);
int launchAllReducePipeline(const mscclppAmdRankView* views, int nviews, int nranks, size_t bytes, int dtype, int op,
                            int nblocks, int nthreads, uint64_t budget, hipStream_t s);
int launchBroadcast(const mscclppAmdRankView* views, int nviews, int nranks, size_t bytes, int root, int nblocks,
                    int nthreads, uint64_t budget, hipStream_t s);
size_t ll16ScratchRequired(int nranks, size_t bytes, int dtype);
size_t ll8ScratchRequired(int nranks, size_t bytes, int dtype);
size_t testLLScratchRequired(int nranks, size_t bytes);
size_t testK2ScratchRequired(int nranks, size_t bytes);
struct BulkGeom;
size_t bulkScratchRequired(int nranks, size_t bytes, size_t maxScratch, BulkGeom* out, int nblocks);
}  // namespace mscclpp_amd

namespace mscclpp_amd {
namespace host {

struct HipError : std::runtime_error {
  hipError_t code;
  HipError(hipError_t c, const char* what) : std::runtime_error(what), code(c) {}
};

#define HIPCHECK(cmd)                                                                               \
  do {                                                                                              \
    hipError_t e_ = (cmd);                                                                          \
    if (e_ != hipSuccess) {                                                                         \
      char buf_[256];                                                                               \
      snprintf(buf_, sizeof(buf_), "%s:%d %s -> %s", __FILE__, __LINE__, #cmd, hipGetErrorString(e_)); \
      throw HipError(e_, buf_);                                                                     \
    }                                                                                               \
  } while (0)

inline thread_local std::string gLastError;

inline int logLevel() {
  static int lvl = [] {
    const char* e = std::getenv("MSCCLPP_LOG_LEVEL");
    if (!e) return 1;
    std::string s(e);
    if (s == "DEBUG" || s == "TRACE") return 3;
    if (s == "INFO") return 2;
    if (s == "WARN") return 1;
    return 0;
  }();
  return lvl;
}

inline void warn(const std::string& m) {
  gLastError = m;
  if (logLevel() >= 1) fprintf(stderr, "[mscclpp_amd WARN] %s\n", m.c_str());
}
inline void info(const std::string& m) {
  if (logLevel() >= 2) fprintf(stderr, "[mscclpp_amd INFO] %s\n", m.c_str());
}

template <typename F>
int guarded(F&& f) {
  try {
    return f();
  } catch (const HipError& e) {
    warn(e.what());
    return ncclUnhandledCudaError;
  } catch (const mscclpp_amd::CudaError& e) {  // a failed HIP runtime call (MSCCLPP_CUDATHROW, gpu_utils.hpp)
    warn(e.what());
    return ncclUnhandledCudaError;
  } catch (const mscclpp_amd::Error& e) {  // the host channel API's errors (core.hpp)
    warn(e.what());
    switch (e.getErrorCode()) {
      case mscclpp_amd::ErrorCode::InvalidUsage: return ncclInvalidUsage;
      case mscclpp_amd::ErrorCode::RemoteError:
      case mscclpp_amd::ErrorCode::Timeout: return ncclRemoteError;
      case mscclpp_amd::ErrorCode::SystemError: return ncclSystemError;
      default: return ncclInternalError;
    }
  } catch (const std::invalid_argument& e) {
    warn(e.what());
    return ncclInvalidArgument;
  } catch (const std::logic_error& e) {  // InvalidUsage (e.g. no selector, null executor)
    warn(e.what());
    return ncclInvalidUsage;
  } catch (const std::exception& e) {
    warn(e.what());
    return ncclInternalError;
  } catch (...) {
    warn("unknown exception");
    return ncclInternalError;
  }
}

inline uint64_t spinBudgetTicks() {
  static uint64_t t = [] {
    const char* e = std::getenv("MSCCLPP_AMD_SPIN_TIMEOUT_MS");
    uint64_t ms = e ? std::strtoull(e, nullptr, 10) : 20000;
    if (ms == 0) ms = 20000;
    return ms * 100000ull;  // s_memrealtime ticks at 100 MHz
  }();
  return t;
}

// MSCCLPP_AMD_BULK_SCRATCH_MB (default 128, the reference's scratch, nccl.cc:180): the bulk scratch
// allocated once at communicator init and never re-allocated; a bucket whose n regions do not fit
// runs in several passes (bulkScratchRequired).
inline size_t bulkScratchInitBytes() {
  const char* e = std::getenv("MSCCLPP_AMD_BULK_SCRATCH_MB");
  size_t mb = e ? std::strtoull(e, nullptr, 10) : 128;
  if (mb < 64) mb = 64;
  return mb << 20;
}

// Uncached device memory (hipDeviceMallocUncached, zeroed) from the process-lifetime pool
// (uncached_pool.cpp: never returned to HIP while the process runs).  freeDevice
// returns a pooled block to the pool and hipFree's anything else, and never throws (destructors
// call it); releaseUncached is false for a pointer the pool does not own.  A release never
// synchronizes (*syncError stays hipSuccess): the block is reused only after the device has drained,
// at the allocation that reuses it (uncached_pool.cpp).
void* allocUncached(size_t bytes);
bool releaseUncached(void* p, hipError_t* syncError) noexcept;
// Fill `bytes` of device memory with `value` and return once the fill has completed on the device
// (own non-blocking stream + synchronize, as the reference's gpuMemset, gpu_utils.cc:274-283).  Every
// set-up fill of memory that a peer, a proxy or a kernel on another stream may touch next goes
// through it: a plain hipMemset is asynchronous to the host, so a host barrier or exchange after it
// orders nothing on the device.
void memsetSync(void* p, int value, size_t bytes);
void freeDevice(void* p) noexcept;
void uncachedPoolStats(size_t* held, size_t* inUse, size_t* freeBytes);
bool isPooledUncached(const void* base);  // `base` is a live block of the pool (an allocation base)

inline int dtypeFromNccl(ncclDataType_t t) {
  switch (t) {
    case ncclFloat16: return MSCCLPP_AMD_F16;
    case ncclBfloat16: return MSCCLPP_AMD_BF16;
    case ncclFloat32: return MSCCLPP_AMD_F32;
    case ncclInt32: return MSCCLPP_AMD_I32;
    case ncclUint32: return MSCCLPP_AMD_U32;
    case ncclFloat8e4m3: return MSCCLPP_AMD_E4M3;  // OCP on gfx950 (datatype_conversion.hpp:29-40)
    case ncclFloat8e5m2: return MSCCLPP_AMD_E5M2;
    case ncclUint8: return MSCCLPP_AMD_U8;  // datatype_conversion.hpp:21-22
    default: return -1;
  }
}
// (element dtype, accumulation dtype) -> reduce-type code; accum < 0 means AUTO = the element type
// (algorithm.cc:47), FP8 may accumulate in half or float (dispatchFp8Accum, common.hpp:89-100).
inline int reduceTypeFromNccl(int ncclDtype, int accum) {
  const int dt = dtypeFromNccl((ncclDataType_t)ncclDtype);
  if (dt < 0 || accum < 0 || accum == ncclDtype) return dt;
  if (dt == MSCCLPP_AMD_E4M3 || dt == MSCCLPP_AMD_E5M2) {
    const int e5 = dt == MSCCLPP_AMD_E5M2;
    if (accum == ncclFloat16) return e5 ? MSCCLPP_AMD_E5M2_ACC_F16 : MSCCLPP_AMD_E4M3_ACC_F16;
    if (accum == ncclFloat32) return e5 ? MSCCLPP_AMD_E5M2_ACC_F32 : MSCCLPP_AMD_E4M3_ACC_F32;
  }
  return -1;  // the reference returns no kernel for other (dtype, accum) pairs
}
inline size_t ncclTypeBytes(ncclDataType_t t) {
  switch (t) {
    case ncclInt8: case ncclUint8: case ncclFloat8e4m3: case ncclFloat8e5m2: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return 0;
  }
}
inline int opFromNccl(ncclRedOp_t op) {
  if (op == ncclSum) return MSCCLPP_AMD_SUM;
  if (op == ncclMin) return MSCCLPP_AMD_MIN;
  return -1;
}

// MSCCLPP_NCCL_SYMMETRIC_MEMORY (env.hpp:101-107, env.cpp:67; any value but "0" is true): every rank
// allocates its communication buffers symmetrically, so a buffer sits at the same offset inside its
// allocation on every rank.  Registration then needs no host exchange for a new buffer inside an
// allocation that is already registered (the reference caches one context per allocation in that
// mode and passes the offset to the kernel, allreduce_fullmesh.cu:206-208, :248-257).
inline bool envSymmetricMemory() {
  const char* e = std::getenv("MSCCLPP_AMD_NCCL_SYMMETRIC_MEMORY");
  if (!e) e = std::getenv("MSCCLPP_NCCL_SYMMETRIC_MEMORY");
  return e && std::string(e) != "0";
}

inline size_t envMaxUserRegs() {
  const char* e = std::getenv("MSCCLPP_AMD_MAX_USER_REGS");
  const long v = e ? std::atol(e) : 0;
  return v > 0 ? (size_t)v : 1024;
}

inline int envAlgo() {  // MSCCLPP_AMD_ALGO, read once
  static const int algo = [] {
    const char* e = std::getenv("MSCCLPP_AMD_ALGO");
    if (!e) return (int)MSCCLPP_AMD_ALGO_AUTO;
    const std::string s(e);
    if (s == "packet") return (int)MSCCLPP_AMD_ALGO_PACKET;
    if (s == "allpair" || s == "allpair_packet") return (int)MSCCLPP_AMD_ALGO_ALLPAIR;
    if (s == "fullmesh") return (int)MSCCLPP_AMD_ALGO_FULLMESH;
    if (s == "rsag") return (int)MSCCLPP_AMD_ALGO_RSAG;
    if (s == "rsag_zc" || s == "rsag_zero_copy") return (int)MSCCLPP_AMD_ALGO_RSAG_ZC;
    if (s == "rsag_pipeline") return (int)MSCCLPP_AMD_ALGO_RSAG_PIPELINE;
    return (int)MSCCLPP_AMD_ALGO_AUTO;
  }();
  return algo;
}

}  // namespace host
}  // namespace mscclpp_amd

using namespace mscclpp_amd;
using namespace mscclpp_amd::host;

namespace mscclpp_amd {
namespace host {
// Process-wide cache of opened IPC handles (gpu_ipc_mem.cc:193-223 keeps one for HIP too): a handle
// is opened once per process however many owners hold it, and closed when the last owner drops
// its reference.  Implemented in core.cpp.
std::shared_ptr<void> openIpcHandle(const hipIpcMemHandle_t& handle);
// An import of a peer's allocation (base, bytes) exported by process `owner` (its processNonce).
// pooled: the owner's uncached pool holds the block for its whole life, so the mapping is kept open
// for the life of this process and reused by later exports of the same block (core.cpp); otherwise
// openIpcHandle.
std::shared_ptr<void> openIpcImport(const hipIpcMemHandle_t& handle, uint64_t owner, uint64_t base, uint64_t bytes,
                                    bool pooled);
uint64_t processNonce();  // random, fixed per process: tells exporters' pools apart
void keptIpcImports(std::vector<std::pair<uint64_t, uint64_t>>* ranges);  // (mapped address, bytes)
size_t releaseKeptIpcImports();  // forget every kept import (mscclppAmdIpcReleaseKept)
size_t liveIpcMappings();
// Drop a reference to a mapping on the closer thread (core.cpp): a close waits for the device to go
// idle, which must not happen on a caller's thread.  pendingMappingReleases = queued or running.
void releaseMappingLater(int device, std::shared_ptr<void> map);
size_t pendingMappingReleases();
uint64_t allocationId(const void* ptr);  // HIP_POINTER_ATTRIBUTE_BUFFER_ID (0 if unknown)
// Tuned configuration (tuning.cpp) for a collective of `bytes` on `nranks` ranks of this device's
// SKU: the algorithm name and launch shape (0 = the algorithm's default); false if none.
// nBlocks value a built-in algorithm's caller passes when it has looked the tuned launch shape up
// itself and found none: use the defaults without looking again.
constexpr int kTunedShapeResolved = -2147483647;
// Generation of the tuned-config store (changes whenever a file is loaded into it).
uint64_t tunedGeneration();
bool tunedConfig(const std::string& collective, int nranks, uint64_t bytes, std::string& algorithm, int& nblocks,
                 int& nthreads, std::string* source = nullptr);
int algoCodeOf(const std::string& name);  // MSCCLPP_AMD_ALGO_* of a default_allreduce_* name, or -1
}  // namespace host
}  // namespace mscclpp_amd

// Every rank's buffer as mapped in this process, plus the references that keep the peers' mappings
// open (entry [rank] is the local pointer and holds no reference).
struct PeerBufs {
  std::array<void*, MSCCLPP_AMD_MAX_RANKS> ptr{};
  std::array<std::shared_ptr<void>, MSCCLPP_AMD_MAX_RANKS> maps{};
  void*& operator[](int r) { return ptr[(size_t)r]; }
  void* operator[](int r) const { return ptr[(size_t)r]; }
};

struct IpcBlob {
  hipIpcMemHandle_t handle;
  uint64_t base;    // allocation base in the owner's address space (cache key)
  uint64_t offset;  // pointer - base
  uint64_t bytes;
  uint64_t owner;   // the exporting process's processNonce()
  uint32_t pooled;  // the allocation is a block of the owner's uncached pool (kept-open import)
  uint32_t pad;
};

// This process's export record of the allocation holding `ptr`.
inline IpcBlob exportBlob(const void* ptr) {
  IpcBlob b{};
  void* base = nullptr;
  size_t sz = 0;
  HIPCHECK(hipMemGetAddressRange((hipDeviceptr_t*)&base, &sz, (hipDeviceptr_t)ptr));
  HIPCHECK(hipIpcGetMemHandle(&b.handle, base));
  b.base = (uint64_t)base;
  b.offset = (uint64_t)((const char*)ptr - (char*)base);
  b.bytes = sz;
  b.owner = processNonce();
  b.pooled = isPooledUncached(base) ? 1u : 0u;
  return b;
}

inline std::shared_ptr<void> importBlob(const IpcBlob& b) {
  return openIpcImport(b.handle, b.owner, b.base, b.bytes, b.pooled != 0);
}

struct ncclComm {
  std::unique_ptr<StarBootstrap> boot;
  // the C++ plugin layer (algorithm.cpp): handle passed to Algorithm::execute, the collection the
  // NCCL entry points select from (nccl.cc:176, :308-314) and the executor for DSL algorithms,
  // created on the first DSL selection (collective: every rank selects the same algorithm)
  std::shared_ptr<mscclpp_amd::Communicator> cxx;
  std::unique_ptr<mscclpp_amd::AlgorithmCollection> algos;
  // the vendor library's communicator for operations this path does not carry (nccl.cc:331-346),
  // present when MSCCLPP_AMD_NCCL_LIB_PATH names librccl (nccl_compat.cpp)
  void* fallback = nullptr;
  hipStream_t errStream = nullptr;  // ncclCommGetAsyncError's reads
  // the copy stream every host-channel Connection of this communicator shares (core.cpp connect);
  // owned by the connections, created by the first one
  std::weak_ptr<void> ipcStream;
  std::mutex ipcStreamMu;
  static constexpr size_t kPipeSemsWords = 3 * 256 + 64;
  uint64_t* pipeSems = nullptr;      // rsag_pipeline's intra-launch counters (3 x 256 + done count)
  std::shared_ptr<mscclpp_amd::Executor> executor;
  void buildAlgorithms();
  // Selection memo of the NCCL entry points (comm.cpp selectAndExecute): the built-in selector's
  // choice and the tuned launch shape per (collective, message size, dtype), valid for one
  // tuned-store generation.  Used only while no user selector is set: a user's selector is asked on
  // every call, as the reference does.
  struct SelMemo {
    const char* coll = nullptr;
    size_t size = 0;
    int dtype = -1;
    uint64_t gen = 0;
    std::shared_ptr<mscclpp_amd::Algorithm> algo;
    int nb = 0, nt = 0;
  };
  std::array<SelMemo, 16> selMemo{};
  std::mutex selMu;
  int rank = 0, nranks = 1, device = 0;
  // LL scratch (two halves, packets), bulk scratch, semaphores, flags, error word
  void* llScratch = nullptr;
  size_t llBytes = 0;
  void* bulkScratch = nullptr;
  size_t bulkBytes = 0;
  uint64_t* tokens = nullptr;
  uint64_t* expected = nullptr;
  uint32_t* flags = nullptr;
  uint32_t* err = nullptr;
  PeerBufs peerLL, peerBulk, peerTok;
  std::array<uint64_t*, MSCCLPP_AMD_MAX_RANKS> peerTokens{};
  // Where a mapping was last used: one event per stream that launched a kernel through it, recorded
  // right after that launch (re-recorded by later launches on the same stream).
  struct UseEvents {
    std::vector<std::pair<hipStream_t, hipEvent_t>> ev;
    // `device`: the communicator's (and the stream's); the event is created there whatever device
    // the calling thread has current
    void record(hipStream_t s, int device) {
      for (auto& e : ev)
        if (e.first == s) {
          HIPCHECK(hipEventRecord(e.second, s));
          return;
        }
      if (ev.size() >= 8) {  // a caller cycling through many streams: forget the uses that completed
        size_t k = 0;
        for (auto& e : ev) {
          if (hipEventQuery(e.second) == hipSuccess) (void)hipEventDestroy(e.second);
          else ev[k++] = e;
        }
        (void)hipGetLastError();
        ev.resize(k);
      }
      int cur = device;
      HIPCHECK(hipGetDevice(&cur));
      if (cur != device) HIPCHECK(hipSetDevice(device));
      hipEvent_t x = nullptr;
      const hipError_t e = hipEventCreateWithFlags(&x, hipEventDisableTiming);
      if (cur != device) (void)hipSetDevice(cur);
      HIPCHECK(e);
      ev.push_back({s, x});
      HIPCHECK(hipEventRecord(x, s));
    }
  };
  // Mappings that queued kernels may still use: each closes (its reference drops) once every event
  // of its last uses has completed -- polled with hipEventQuery at the next call (flushRetired), so
  // no call waits for another stream's work and none synchronizes the device (VERDICT r4 item 4;
  // the reference's context cache never synchronizes either, algorithm.cc:52-60).
  struct Retired {
    std::vector<std::shared_ptr<void>> maps;
    UseEvents uses;
  };
  std::vector<Retired> retired;
  // user registrations whose pointers the current call handed to its kernel (recordUses after launch)
  std::vector<UseEvents*> touched;
  std::mutex mu;

  // Exchange an IPC handle of the allocation holding `ptr` and return every rank's pointer as mapped
  // here (collective).  Mappings come from the process-wide cache (openIpcHandle), so a peer buffer
  // mapped by several owners is opened once; a peer that freed an allocation and got a new one at
  // the same address sends a new handle, which maps afresh.
  PeerBufs exchange(void* ptr) {
    const IpcBlob mine = exportBlob(ptr);
    if (std::getenv("MSCCLPP_AMD_DEBUG_IPC"))
      std::fprintf(stderr, "ipc rank %d export ptr %p base %llx bytes %llu id %llu pooled %u\n", rank, ptr,
                   (unsigned long long)mine.base, (unsigned long long)mine.bytes,
                   (unsigned long long)allocationId((void*)mine.base), mine.pooled);
    info("rank " + std::to_string(rank) + ": got ipc handle, all-gather");
    std::vector<IpcBlob> all(nranks);
    boot->allGather(&mine, all.data(), sizeof(IpcBlob));
    PeerBufs res;
    for (int r = 0; r < nranks; ++r) {
      if (r == rank) {
        res[r] = ptr;
        continue;
      }
      res.maps[(size_t)r] = importBlob(all[r]);
      res[r] = (char*)res.maps[(size_t)r].get() + all[r].offset;
    }
    if (std::getenv("MSCCLPP_AMD_DEBUG_IPC")) {  // one line per peer: what was imported and where
      for (int r = 0; r < nranks; ++r) {
        if (r == rank) continue;
        std::string hex;
        const unsigned char* h = reinterpret_cast<const unsigned char*>(&all[r].handle);
        for (size_t i = 0; i < sizeof(all[r].handle); ++i) {
          char b[3];
          std::snprintf(b, sizeof b, "%02x", h[i]);
          hex += b;
        }
        std::fprintf(stderr, "ipc rank %d peer %d base %llx bytes %llu handle %s mapped %p\n", rank, r,
                     (unsigned long long)all[r].base, (unsigned long long)all[r].bytes, hex.c_str(), res.maps[(size_t)r].get());
      }
    }
    return res;
  }

  // Close the retired mappings whose last uses have completed; the others wait for a later call.
  // Never blocks.
  void flushRetired() {
    size_t keep = 0;
    for (size_t i = 0; i < retired.size(); ++i) {
      bool done = true;
      for (auto& e : retired[i].uses.ev) {
        const hipError_t q = hipEventQuery(e.second);
        if (q == hipErrorNotReady) {
          done = false;
          break;
        }
        if (q != hipSuccess) (void)hipGetLastError();  // a failed event cannot hold a mapping open
      }
      if (done) {
        for (auto& e : retired[i].uses.ev) (void)hipEventDestroy(e.second);
        retired[i].uses.ev.clear();
        for (auto& m : retired[i].maps) releaseMappingLater(device, std::move(m));
        retired[i].maps.clear();
      } else if (keep != i) {
        retired[keep++] = std::move(retired[i]);
      } else {
        ++keep;
      }
    }
    retired.resize(keep);
  }

  // Every retired mapping, whatever is still queued: only after a device synchronize (teardown).
  void clearRetired() {
    for (auto& r : retired)
      for (auto& e : r.uses.ev) (void)hipEventDestroy(e.second);
    retired.clear();
  }

  static bool capturing(hipStream_t stream) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    return stream && hipStreamIsCapturing(stream, &st) == hipSuccess && st != hipStreamCaptureStatusNone;
  }

  // After a launch on `stream`: the registrations it used record their use there.  Under capture
  // nothing is recorded -- those registrations are pinned (never retired while a graph may replay).
  void recordUses(hipStream_t stream) {
    if (touched.empty()) return;  // the LL paths register nothing: no extra host call per launch
    if (!capturing(stream))
      for (UseEvents* u : touched) u->record(stream, device);
    touched.clear();
  }

  // Grow a scratch region collectively (every rank calls with the same size at the same call).
  // The outgrown buffer is kept allocated until the communicator is destroyed: freeing it let the
  // allocator hand its address range to the new buffer, and peers that imported the new buffer's
  // IPC handle then wrote through a mapping of the OLD memory (8 processes, one GPU: after the
  // bulk scratch grew 64 -> 128 MiB, two ranks' peers wrote the pipeline's stages into the old
  // buffer, tools/multi_rank_check.py).  Growth is geometric, so what is kept is at most the final size.
  std::vector<void*> outgrown;
  //
  // Growth synchronizes the device and allocates, so it cannot happen inside a HIP graph capture:
  // a call that would grow while `stream` captures fails with ncclInvalidUsage instead (run the
  // same call once eagerly before capturing, and the scratch is already large enough).
  void ensure(void*& buf, size_t& have, PeerBufs& peers, size_t need, hipStream_t stream = nullptr) {
    if (need <= have) return;
    if (stream) {
      hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
      if (hipStreamIsCapturing(stream, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)
        throw std::logic_error("scratch must grow to " + std::to_string(need) +
                               " bytes, which cannot happen while the stream is capturing a graph: run this call "
                               "once before capture");
    }
    size_t want = have ? have : (size_t)64 << 20;
    while (want < need) want *= 2;
    HIPCHECK(hipDeviceSynchronize());
    boot->barrier();  // every rank has drained its previous use of the old buffers
    peers = PeerBufs();  // our mappings of the peers' old buffers close here
    if (buf) outgrown.push_back(buf);
    buf = allocUncached(want);
    have = want;
    peers = exchange(buf);
    boot->barrier();
    info("rank " + std::to_string(rank) + " scratch grown to " + std::to_string(want));
  }

  // Peer pointers of a user buffer (the bulk kernels write results straight into every peer's
  // output, allreduce_fullmesh.cu:110-113; zero-copy reads the peers' inputs).  Cached per local
  // allocation like the reference's per-buffer context cache (algorithm.cc:52-60): a repeated call on
  // the same buffer costs no host round trip.  As in the reference, every rank must pass its
  // matching buffer when a buffer is first used.
  //  * The allocation is identified by (base, size, HIP buffer id): a buffer freed and re-allocated
  //    at the same address is a new allocation, registered afresh, and its old registration retired.
  //  * At most kMaxUserRegs allocations stay registered; the least recently used one is retired
  //    beyond that (every rank sees the same sequence of buffers, so every rank evicts the same).
  //  * Retired mappings close once the kernels that used them have completed (the events recorded
  //    after those launches, flushRetired), never under a running kernel and with no synchronize.
  //  * A registration used while its stream is capturing a HIP graph is pinned: the graph keeps
  //    the peer pointers in its kernel arguments, so evicting it (and closing the mappings) would
  //    leave every later replay writing through closed mappings.  Pinned entries are never evicted
  //    (the cap then only bounds the unpinned ones); capture happens in the same calls on every
  //    rank, so every rank pins the same.
  //  * A registration made for the caller (Communicator::registerMemory, mscclppAmdCommRegisterBuffer)
  //    is pinned too: the caller keeps the raw peer pointers (an algorithm plugin's context holds
  //    them for good), so no later eviction may close them.
  //  * Pinned entries are released only by dropUserRegistrations (mscclppAmdCommDeregisterAll), which
  //    must not run while a graph that captured them is still replayed, or when the address is
  //    re-used by a new allocation (the old one was freed, so its pointers were dead already).
  // kMaxUserRegs: 1024 by default, MSCCLPP_AMD_MAX_USER_REGS sets it.  The reference's context cache
  // has no bound (algorithm.cc:52-60); a small one made a caller cycling through more buckets
  // re-register on every call -- a host exchange, and, with the device busy, a wait for the close of
  // the same handle still in flight (openIpcHandle; 2.8 s behind a 2.8 s kernel in
  // tests/test_no_device_sync_gpu.py).  A bound is still kept: each registration keeps the peers'
  // allocations mapped, so a peer's freed buffer stays held until its registration is retired.
  const size_t kMaxUserRegs = envMaxUserRegs();
  struct UserReg {
    uint64_t bufferId = 0;
    uint64_t lastUse = 0;
    bool pinned = false;  // used under stream capture
    PeerBufs bases;
    UseEvents uses;
    std::map<uint64_t, std::array<void*, MSCCLPP_AMD_MAX_RANKS>> byOffset;
  };
  std::map<std::pair<uint64_t, uint64_t>, UserReg> userRegs;
  uint64_t useClock = 0;
  bool symmetricMemory = envSymmetricMemory();
  // host all-gathers the registration path made: allocations exchanged, offsets exchanged
  uint64_t allocExchanges = 0, offsetExchanges = 0;

  void retireReg(std::map<std::pair<uint64_t, uint64_t>, UserReg>::iterator it) {
    if (it->second.pinned)
      info("rank " + std::to_string(rank) + ": pinned registration of allocation " +
           std::to_string(it->first.first) + " retired (its address now belongs to a new allocation)");
    Retired r;
    for (auto& m : it->second.bases.maps)
      if (m) r.maps.push_back(std::move(m));
    r.uses = std::move(it->second.uses);
    for (auto t = touched.begin(); t != touched.end();)  // not recorded for a launch any more
      t = *t == &it->second.uses ? touched.erase(t) : t + 1;
    if (!r.maps.empty() || !r.uses.ev.empty()) retired.push_back(std::move(r));
    userRegs.erase(it);
  }

  std::array<void*, MSCCLPP_AMD_MAX_RANKS> registerOutput(void* out, hipStream_t stream = nullptr, bool pin = false) {
    void* base = nullptr;
    size_t sz = 0;
    HIPCHECK(hipMemGetAddressRange((hipDeviceptr_t*)&base, &sz, (hipDeviceptr_t)out));
    const uint64_t bid = allocationId(base);
    const auto key = std::make_pair((uint64_t)base, (uint64_t)sz);
    auto it = userRegs.find(key);
    if (it != userRegs.end() && it->second.bufferId != bid) {
      retireReg(it);  // the address now belongs to another allocation
      it = userRegs.end();
    }
    if (it == userRegs.end()) {
      size_t unpinned = 0;
      for (const auto& e : userRegs) unpinned += e.second.pinned ? 0 : 1;
      if (unpinned >= kMaxUserRegs) {
        auto lru = userRegs.end();
        for (auto j = userRegs.begin(); j != userRegs.end(); ++j)
          if (!j->second.pinned && (lru == userRegs.end() || j->second.lastUse < lru->second.lastUse)) lru = j;
        retireReg(lru);
      }
      UserReg reg;
      reg.bufferId = bid;
      reg.bases = exchange(base);  // collective: every rank registers its matching buffer now
      ++allocExchanges;
      it = userRegs.emplace(key, std::move(reg)).first;
    }
    UserReg& reg = it->second;
    reg.lastUse = ++useClock;
    if (pin) reg.pinned = true;
    if (stream) {
      hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
      if (hipStreamIsCapturing(stream, &cs) == hipSuccess && cs == hipStreamCaptureStatusActive) reg.pinned = true;
    }
    const uint64_t off = (uint64_t)((char*)out - (char*)base);
    auto pit = reg.byOffset.find(off);
    if (pit == reg.byOffset.end()) {
      // The offset of `out` inside its allocation may differ between ranks: exchange offsets (cheap)
      // to build exact pointers -- unless the application declared symmetric allocation, where it
      // is the same on every rank and this call stays local.
      std::vector<uint64_t> offs(nranks, off);
      if (!symmetricMemory) {
        boot->allGather(&off, offs.data(), sizeof(off));
        ++offsetExchanges;
      }
      std::array<void*, MSCCLPP_AMD_MAX_RANKS> res{};
      for (int r = 0; r < nranks; ++r) res[r] = (r == rank) ? out : (char*)reg.bases[r] + offs[r];
      pit = reg.byOffset.emplace(off, res).first;
    }
    const auto res = pit->second;
    touched.push_back(&reg.uses);
    flushRetired();
    return res;
  }

  // Broadcast: every rank all-gathers an IPC handle (root: its send buffer; others: their receive
  // buffer, only so the call stays collective) and opens only the root's.  Done on every call: the
  // root's buffer is not known to the other ranks in advance, so a per-buffer cache could not stay
  // consistent across ranks.
  int broadcast(const void* send, void* recv, size_t bytes, int root, int nblocks, int nthreads, hipStream_t stream) {
    std::lock_guard<std::mutex> lk(mu);
    const void* mine = rank == root ? send : recv;
    const IpcBlob blob = exportBlob(mine);
    std::vector<IpcBlob> all(nranks);
    boot->allGather(&blob, all.data(), sizeof(IpcBlob));
    mscclppAmdRankView v = baseView(rank == root ? send : recv, recv);
    if (rank != root) {
      // the mapping stays referenced until a later broadcast from the same root replaces it (and
      // is then retired: the kernel below may still be queued).  A mapping used under stream
      // capture is kept until dropUserRegistrations instead: the graph's replays read through it.
      auto m = importBlob(all[root]);
      auto& slot = bcastMaps[(size_t)root];
      bool& captured = bcastCaptured[(size_t)root];  // sticky while the same mapping stays in the slot
      if (slot && slot != m) {
        if (captured) {
          bcastPinned.push_back(std::move(slot));
        } else {
          Retired r;
          r.maps.push_back(std::move(slot));
          r.uses = std::move(bcastUses[(size_t)root]);
          retired.push_back(std::move(r));
        }
        bcastUses[(size_t)root] = UseEvents();
        captured = false;
      }
      slot = m;
      hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
      if (stream && hipStreamIsCapturing(stream, &cs) == hipSuccess && cs == hipStreamCaptureStatusActive)
        captured = true;
      v.peerInput[root] = (char*)m.get() + all[root].offset;
    }
    const int rc = launchBroadcast(&v, 1, nranks, bytes, root, nblocks, nthreads, spinBudgetTicks(), stream);
    if (rank != root && rc == 0 && !capturing(stream)) bcastUses[(size_t)root].record(stream, device);
    flushRetired();
    return rc;
  }
  std::array<std::shared_ptr<void>, MSCCLPP_AMD_MAX_RANKS> bcastMaps;
  std::array<UseEvents, MSCCLPP_AMD_MAX_RANKS> bcastUses;  // the launches that read bcastMaps[root]
  std::array<bool, MSCCLPP_AMD_MAX_RANKS> bcastCaptured{};  // bcastMaps[root] used under capture
  std::vector<std::shared_ptr<void>> bcastPinned;             // replaced, but a graph may read them

  // Drop every cached mapping of peers' user buffers (collective).  Scratch, token and flag
  // mappings stay.  After this, the next use of any buffer registers it afresh.
  void dropUserRegistrations() {
    HIPCHECK(hipDeviceSynchronize());
    boot->barrier();  // no rank still runs a kernel that uses a mapping being closed
    while (!userRegs.empty()) retireReg(userRegs.begin());
    for (auto& m : bcastMaps) m.reset();
    for (auto& u : bcastUses)
      for (auto& e : u.ev) (void)hipEventDestroy(e.second);
    bcastUses = {};
    bcastCaptured = {};
    bcastPinned.clear();
    clearRetired();
    boot->barrier();
  }

  // The tuned launch shape of `algo` for this message, when the caller left the shape open and the
  // tuned entry names the same algorithm.
  void applyTunedShape(const char* coll, int algo, size_t bytes, int& nblocks, int& nthreads) {
    if (nblocks > 0 || nthreads > 0) return;
    std::string name;
    int nb = 0, nt = 0;
    if (tunedConfig(coll, nranks, bytes, name, nb, nt) && algoCodeOf(name) == algo) {
      nblocks = nb;
      nthreads = nt;
    }
  }

  mscclppAmdRankView baseView(const void* in, void* out) {
    mscclppAmdRankView v{};
    v.input = in;
    v.output = out;
    v.tokens = tokens;
    v.expected = expected;
    v.flags = flags;
    v.err = err;
    v.rank = rank;
    for (int r = 0; r < nranks; ++r) v.peerTokens[r] = peerTokens[r];
    return v;
  }

  int allReduce(const void* in, void* out, size_t bytes, int dtype, int op, int algo, int nblocks, int nthreads,
                hipStream_t stream) {
    std::lock_guard<std::mutex> lk(mu);
    touched.clear();
    const int rc = allReduceLaunch(in, out, bytes, dtype, op, algo, nblocks, nthreads, stream);
    recordUses(stream);
    return rc;
  }

  int allReduceLaunch(const void* in, void* out, size_t bytes, int dtype, int op, int algo, int nblocks, int nthreads,
                      hipStream_t stream) {
    if (algo == MSCCLPP_AMD_ALGO_AUTO) algo = envAlgo();
    if (algo == MSCCLPP_AMD_ALGO_AUTO) {
      algo = mscclppAmdSelectAlgo(nranks, bytes, dtype);
      applyTunedShape("allreduce", algo, bytes, nblocks, nthreads);
    }
    // the pipelined RS+AG carries 2- and 4-byte types only; others take fullmesh, which carries all
    if (algo == MSCCLPP_AMD_ALGO_RSAG_PIPELINE && dtype != MSCCLPP_AMD_F16 && dtype != MSCCLPP_AMD_BF16 &&
        dtype != MSCCLPP_AMD_F32 && dtype != MSCCLPP_AMD_I32 && dtype != MSCCLPP_AMD_U32)
      algo = MSCCLPP_AMD_ALGO_FULLMESH;
    mscclppAmdRankView v = baseView(in, out);
    if (algo == MSCCLPP_AMD_ALGO_PACKET || algo == MSCCLPP_AMD_ALGO_ALLPAIR || algo == MSCCLPP_AMD_ALGO_TEST_K6 ||
        algo == MSCCLPP_AMD_ALGO_TEST_K7 || algo == MSCCLPP_AMD_ALGO_TEST_K2) {
      const size_t need = algo == MSCCLPP_AMD_ALGO_PACKET    ? ll16ScratchRequired(nranks, bytes, dtype)
                          : algo == MSCCLPP_AMD_ALGO_ALLPAIR ? ll8ScratchRequired(nranks, bytes, dtype)
                          : algo == MSCCLPP_AMD_ALGO_TEST_K2 ? testK2ScratchRequired(nranks, bytes)
                                                             : testLLScratchRequired(nranks, bytes);
      if (need == 0) return ncclInvalidUsage;
      ensure(llScratch, llBytes, peerLL, need, stream);
      v.scratch = llScratch;
      v.scratchBytes = llBytes;
      for (int r = 0; r < nranks; ++r) v.peerScratch[r] = peerLL[r];
      return launchAllReduceLL(algo, &v, 1, nranks, bytes, dtype, op, nblocks, nthreads, spinBudgetTicks(), stream);
    }
    if (algo == MSCCLPP_AMD_ALGO_FULLMESH || algo == MSCCLPP_AMD_ALGO_RSAG) {
      // the scratch allocated at init bounds a pass; larger buckets take several passes
      size_t need = bytes + 16 * (size_t)nranks * 64;
      const size_t cap = bulkBytes;
      if (need > cap) need = cap;
      ensure(bulkScratch, bulkBytes, peerBulk, need, stream);
      v.scratch = bulkScratch;
      v.scratchBytes = bulkBytes;
      for (int r = 0; r < nranks; ++r) v.peerScratch[r] = peerBulk[r];
      auto outs = registerOutput(out, stream);
      for (int r = 0; r < nranks; ++r) v.peerOutput[r] = outs[r];
      return launchAllReduceBulk(algo, &v, 1, nranks, bytes, dtype, op, nblocks, nthreads, spinBudgetTicks(), stream);
    }
    if (algo == MSCCLPP_AMD_ALGO_TEST_K5) {
      if (in != out) {
        warn("mscclpp-test kernel 5 runs in place (sendbuff == recvbuff)");
        return ncclInvalidUsage;
      }
      auto bufs = registerOutput(out, stream);
      for (int r = 0; r < nranks; ++r) v.peerOutput[r] = bufs[r];
      return launchAllReduceBulk(algo, &v, 1, nranks, bytes, dtype, op, nblocks, nthreads, spinBudgetTicks(), stream);
    }
    if (algo == MSCCLPP_AMD_ALGO_RSAG_PIPELINE) {
      // every remote store lands in the bulk scratch: no user-buffer registration at all
      size_t need = 2 * bytes + 16 * (size_t)nranks * 64;
      if (need > bulkBytes) need = bulkBytes;  // fewer stages, never a re-allocation
      ensure(bulkScratch, bulkBytes, peerBulk, need, stream);
      v.scratch = bulkScratch;
      v.scratchBytes = bulkBytes;
      for (int r = 0; r < nranks; ++r) v.peerScratch[r] = peerBulk[r];
      if (!pipeSems) {  // counters must start at zero; each launch leaves them at zero (allreduce_bulk.hip)
        HIPCHECK(hipMalloc((void**)&pipeSems, kPipeSemsWords * sizeof(uint64_t)));
        HIPCHECK(hipMemset(pipeSems, 0, kPipeSemsWords * sizeof(uint64_t)));
      }
      v.pipeSems = pipeSems;
      return launchAllReducePipeline(&v, 1, nranks, bytes, dtype, op, nblocks, nthreads, spinBudgetTicks(), stream);
    }
    if (algo == MSCCLPP_AMD_ALGO_RSAG_ZC) {
      // zero-copy: peers' inputs and outputs are mapped once per buffer (the reference registers
      // both as remote memories, allreduce_rsag_zero_copy.cu:25-27); no scratch
      auto outs = registerOutput(out, stream);
      auto ins = registerOutput(const_cast<void*>(in), stream);
      for (int r = 0; r < nranks; ++r) {
        v.peerOutput[r] = outs[r];
        v.peerInput[r] = ins[r];
      }
      return launchAllReduceBulk(algo, &v, 1, nranks, bytes, dtype, op, nblocks, nthreads, spinBudgetTicks(), stream);
    }
    return ncclInvalidArgument;
  }

  // ReduceScatter (mode 1) / AllGather (mode 2) through the bulk all-pairs kernel; `bytes` is the
  // per-rank block (recvcount / sendcount bytes).
  int bulkCollective(int mode, const void* in, void* out, size_t blockBytes, int dtype, int op, int algo, int nblocks,
                     int nthreads, hipStream_t stream) {
    std::lock_guard<std::mutex> lk(mu);
    touched.clear();
    const int rc = bulkCollectiveLaunch(mode, in, out, blockBytes, dtype, op, algo, nblocks, nthreads, stream);
    recordUses(stream);
    return rc;
  }

  int bulkCollectiveLaunch(int mode, const void* in, void* out, size_t blockBytes, int dtype, int op, int algo,
                           int nblocks, int nthreads, hipStream_t stream) {
    if (blockBytes % 16) {
      warn("ReduceScatter/AllGather blocks must be a multiple of 16 bytes on this path");
      return ncclInvalidUsage;
    }
    const size_t total = blockBytes * nranks;
    mscclppAmdRankView v = baseView(in, out);
    size_t need = total + 16 * (size_t)nranks * 64;
    const size_t cap = bulkBytes;
    if (need > cap) need = cap;
    ensure(bulkScratch, bulkBytes, peerBulk, need, stream);
    v.scratch = bulkScratch;
    v.scratchBytes = bulkBytes;
    for (int r = 0; r < nranks; ++r) v.peerScratch[r] = peerBulk[r];
    if (mode == 2) {
      auto outs = registerOutput(out, stream);
      for (int r = 0; r < nranks; ++r) v.peerOutput[r] = outs[r];
    } else {
      for (int r = 0; r < nranks; ++r) v.peerOutput[r] = out;  // unused by ReduceScatter
    }
    if (algo != MSCCLPP_AMD_ALGO_RSAG) algo = MSCCLPP_AMD_ALGO_FULLMESH;
    return launchCollectiveBulk(mode, algo, &v, 1, nranks, total, dtype, op, nblocks, nthreads, spinBudgetTicks(),
                                stream);
  }

  void destroy() {
    (void)hipDeviceSynchronize();
    for (auto& m : selMemo) m = SelMemo();
    algos.reset();
    executor.reset();
    if (boot) {
      try {
        boot->barrier();
      } catch (...) {
      }
    }
    for (auto& kv : userRegs)
      for (auto& e : kv.second.uses.ev) (void)hipEventDestroy(e.second);
    userRegs.clear();
    touched.clear();
    for (auto& m : bcastMaps) m.reset();
    for (auto& u : bcastUses)
      for (auto& e : u.ev) (void)hipEventDestroy(e.second);
    bcastUses = {};
    bcastPinned.clear();
    peerLL = peerBulk = peerTok = PeerBufs();
    clearRetired();
    freeDevice(llScratch);
    freeDevice(bulkScratch);
    for (void* p : outgrown) freeDevice(p);
    outgrown.clear();
    freeDevice(tokens);
    if (expected) (void)hipFree(expected);
    if (flags) (void)hipFree(flags);
    if (err) (void)hipFree(err);
    if (errStream) (void)hipStreamDestroy(errStream);
    if (pipeSems) (void)hipFree(pipeSems);
    pipeSems = nullptr;
    errStream = nullptr;
    llScratch = bulkScratch = nullptr;
    tokens = expected = nullptr;
    flags = err = nullptr;
  }
};

// ---- vendor NCCL fallback (nccl_compat.cpp) --------------------------------------------------
namespace mscclpp_amd {
namespace host {
struct VendorNccl {
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*CommFinalize)(ncclComm_t) = nullptr;
  ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, void*) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, void*) = nullptr;
  ncclResult_t (*ReduceScatter)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, void*) = nullptr;
  ncclResult_t (*Broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, void*) = nullptr;
  ncclResult_t (*Reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, int, ncclComm_t, void*) = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, void*) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, void*) = nullptr;
  ncclResult_t (*AllToAll)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, void*) = nullptr;
  ncclResult_t (*AllToAllv)(const void*, const size_t[], const size_t[], void*, const size_t[], const size_t[],
                            ncclDataType_t, ncclComm_t, void*) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  ncclResult_t (*GroupSimulateEnd)(ncclSimInfo_t*) = nullptr;
  ncclResult_t (*RedOpCreatePreMulSum)(ncclRedOp_t*, void*, ncclDataType_t, ncclScalarResidence_t, ncclComm_t) = nullptr;
  ncclResult_t (*RedOpDestroy)(ncclRedOp_t, ncclComm_t) = nullptr;
};
// The vendor library named by MSCCLPP_AMD_NCCL_LIB_PATH (or MSCCLPP_NCCL_LIB_PATH), or null.
const VendorNccl* vendorNccl();
// MSCCLPP_AMD_FORCE_NCCL_FALLBACK_OPERATION ("all" or a comma list of allreduce, allgather,
// reducescatter, broadcast) names `op`.
bool forcedFallback(const char* op);
// ncclCommInitRank with the bootstrap's connect / receive timeout given (ncclCommInitRank takes it
// from MSCCLPP_AMD_BOOTSTRAP_TIMEOUT_S); commId is the 128-byte unique id.  Returns an ncclResult_t.
int commInitRank(ncclComm_t* comm, int nranks, const void* commId, int rank, int timeoutSec);
void initFallbackComm(ncclComm* c);                 // collective over c's bootstrap
void destroyFallbackComm(ncclComm* c, bool abort);
}  // namespace host
}  // namespace mscclpp_amd

