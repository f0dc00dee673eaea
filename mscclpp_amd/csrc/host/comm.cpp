// Host runtime + C ABI of libmscclpp_amd.so.
//
//  * memory helpers        -- GpuBuffer / uncached allocation (reference gpu_utils.cc:139-147) and
//                             the flag buffer (algorithm.cc:251-268)
//  * AllReduce launcher     -- explicit rank views -> LL16 / LL8 / bulk kernels
//  * algorithm selector     -- algorithm_selector.cc:91-139 restated for gfx950 + xGMI
//  * ncclComm + NCCL ABI    -- nccl.cc:187-905: bootstrap, IPC-mapped scratch and semaphores,
//                             per-buffer registration cache (algorithm.cc:42-68 context cache)
// Every C entry point catches C++ exceptions and returns an ncclResult_t (SURVEY §8b "Errors").
#include "comm_internal.hpp"

// =============================================================================================
// C ABI: memory, microbench, launcher, selector
// =============================================================================================
extern "C" {

int mscclppAmdMallocUncached(void** ptr, size_t bytes) {
  return guarded([&] {
    if (!ptr || !bytes) return (int)ncclInvalidArgument;
    *ptr = allocUncached(bytes);
    return (int)ncclSuccess;
  });
}

int mscclppAmdMalloc(void** ptr, size_t bytes) {
  return guarded([&] {
    if (!ptr || !bytes) return (int)ncclInvalidArgument;
    HIPCHECK(hipMalloc(ptr, bytes));
    return (int)ncclSuccess;
  });
}

int mscclppAmdFree(void* ptr) {
  return guarded([&] {
    hipError_t syncErr = hipSuccess;
    if (ptr && !releaseUncached(ptr, &syncErr)) HIPCHECK(hipFree(ptr));
    HIPCHECK(syncErr);
    return (int)ncclSuccess;
  });
}

int mscclppAmdIpcStats(size_t* openMappings, size_t* keptImports) {
  return guarded([&] {
    std::vector<std::pair<uint64_t, uint64_t>> kept;
    keptIpcImports(&kept);
    if (openMappings) *openMappings = liveIpcMappings();
    if (keptImports) *keptImports = kept.size();
    return (int)ncclSuccess;
  });
}

int mscclppAmdIpcReleaseKept(size_t* released) {
  return guarded([&] {
    HIPCHECK(hipDeviceSynchronize());  // no queued kernel may still read through a mapping closed here
    const size_t n = releaseKeptIpcImports();
    if (released) *released = n;
    return (int)ncclSuccess;
  });
}

int mscclppAmdIpcKeptRanges(uint64_t* addrs, uint64_t* bytes, size_t cap, size_t* n) {
  return guarded([&] {
    std::vector<std::pair<uint64_t, uint64_t>> kept;
    keptIpcImports(&kept);
    for (size_t i = 0; i < kept.size() && i < cap; ++i) {
      if (addrs) addrs[i] = kept[i].first;
      if (bytes) bytes[i] = kept[i].second;
    }
    if (n) *n = kept.size();
    return (int)ncclSuccess;
  });
}

int mscclppAmdFlagsInit(uint32_t* flags, void* stream) {
  return guarded([&] {
    if (!flags) return (int)ncclInvalidArgument;
    std::vector<uint32_t> ones(MSCCLPP_AMD_FLAG_SLOTS, 1u);
    HIPCHECK(hipMemcpyAsync(flags, ones.data(), ones.size() * 4, hipMemcpyHostToDevice, (hipStream_t)stream));
    HIPCHECK(hipStreamSynchronize((hipStream_t)stream));
    return (int)ncclSuccess;
  });
}

int mscclppAmdAllReduceLaunch(int algo, const mscclppAmdRankView* views, int nviews, int nranks, size_t bytes,
                              int dtype, int op, int nblocks, int nthreads, uint64_t budgetTicks, void* stream) {
  return guarded([&] {
    if (!views || nviews < 1 || nranks < 2 || nranks > MSCCLPP_AMD_MAX_RANKS || bytes == 0) return (int)ncclInvalidArgument;
    if (nviews != 1 && nviews != nranks) return (int)ncclInvalidArgument;
    if (dtype < 0 || dtype >= MSCCLPP_AMD_NUM_DTYPES || op < 0 || op > MSCCLPP_AMD_MIN) return (int)ncclInvalidArgument;
    if (algo == MSCCLPP_AMD_ALGO_AUTO) algo = mscclppAmdSelectAlgo(nranks, bytes, dtype);
    if (budgetTicks == 0) budgetTicks = spinBudgetTicks();
    // validate every pointer the kernel will dereference before launching (a fault here would
    // take the GPU down; a bad argument must come back as ncclInvalidArgument instead)
    const bool k5 = algo == MSCCLPP_AMD_ALGO_TEST_K5;
    const bool zc = algo == MSCCLPP_AMD_ALGO_RSAG_ZC || k5;  // no scratch: peers' user buffers directly
    const bool bulk = algo == MSCCLPP_AMD_ALGO_FULLMESH || algo == MSCCLPP_AMD_ALGO_RSAG || zc;
    if (algo == MSCCLPP_AMD_ALGO_RSAG_PIPELINE) {
      for (int i = 0; i < nviews; ++i) {
        const mscclppAmdRankView& v = views[i];
        if (!v.input || !v.output || !v.scratch || !v.pipeSems || !v.tokens || !v.expected || !v.err)
          return (int)ncclInvalidArgument;
        for (int q = 0; q < nranks; ++q)
          if (!v.peerScratch[q] || !v.peerTokens[q]) return (int)ncclInvalidArgument;
      }
      return launchAllReducePipeline(views, nviews, nranks, bytes, dtype, op, nblocks, nthreads, budgetTicks,
                                     (hipStream_t)stream);
    }
    const bool ll = algo == MSCCLPP_AMD_ALGO_PACKET || algo == MSCCLPP_AMD_ALGO_ALLPAIR ||
                    algo == MSCCLPP_AMD_ALGO_TEST_K6 || algo == MSCCLPP_AMD_ALGO_TEST_K7 ||
                    algo == MSCCLPP_AMD_ALGO_TEST_K2;
    unsigned seen = 0;
    for (int i = 0; i < nviews; ++i) {
      const mscclppAmdRankView& v = views[i];
      if (v.rank < 0 || v.rank >= nranks || (seen >> v.rank) & 1u) return (int)ncclInvalidArgument;
      seen |= 1u << v.rank;
      if (!v.input || !v.output || !v.flags || !v.err) return (int)ncclInvalidArgument;
      if (ll && ((uintptr_t)v.flags % 16)) return (int)ncclInvalidArgument;  // 16-byte flag refresh
      if (!zc && (!v.scratch || v.scratchBytes == 0)) return (int)ncclInvalidArgument;
      for (int q = 0; q < nranks; ++q) {
        if (!zc && !v.peerScratch[q]) return (int)ncclInvalidArgument;
        if (bulk && (!v.peerOutput[q] || !v.peerTokens[q])) return (int)ncclInvalidArgument;
        if (zc && !k5 && !v.peerInput[q]) return (int)ncclInvalidArgument;
      }
      if (bulk && (!v.tokens || !v.expected)) return (int)ncclInvalidArgument;
    }
    if (ll)
      return launchAllReduceLL(algo, views, nviews, nranks, bytes, dtype, op, nblocks, nthreads, budgetTicks,
                               (hipStream_t)stream);
    if (bulk)
      return launchAllReduceBulk(algo, views, nviews, nranks, bytes, dtype, op, nblocks, nthreads, budgetTicks,
                                 (hipStream_t)stream);
    return (int)ncclInvalidArgument;
  });
}

int mscclppAmdCollectiveLaunch(int coll, int algo, const mscclppAmdRankView* views, int nviews, int nranks,
                               size_t bytes, int dtype, int op, int nblocks, int nthreads, uint64_t budgetTicks,
                               void* stream) {
  if (coll == 0)
    return mscclppAmdAllReduceLaunch(algo, views, nviews, nranks, bytes, dtype, op, nblocks, nthreads, budgetTicks,
                                     stream);
  return guarded([&] {
    if (!views || nviews < 1 || nranks < 2 || nranks > MSCCLPP_AMD_MAX_RANKS || bytes == 0) return (int)ncclInvalidArgument;
    if (nviews != 1 && nviews != nranks) return (int)ncclInvalidArgument;
    if (coll != 1 && coll != 2) return (int)ncclInvalidArgument;
    for (int i = 0; i < nviews; ++i) {
      const mscclppAmdRankView& v = views[i];
      if (!v.input || !v.output || !v.scratch || !v.tokens || !v.expected || !v.err) return (int)ncclInvalidArgument;
      for (int q = 0; q < nranks; ++q)
        if (!v.peerScratch[q] || !v.peerTokens[q] || !v.peerOutput[q]) return (int)ncclInvalidArgument;
    }
    return launchCollectiveBulk(coll, algo, views, nviews, nranks, bytes, dtype, op, nblocks, nthreads,
                                budgetTicks ? budgetTicks : spinBudgetTicks(), (hipStream_t)stream);
  });
}

size_t mscclppAmdScratchRequired(int algo, int nranks, size_t bytes, int dtype) {
  if (algo == MSCCLPP_AMD_ALGO_PACKET) return ll16ScratchRequired(nranks, bytes, dtype);
  if (algo == MSCCLPP_AMD_ALGO_ALLPAIR) return ll8ScratchRequired(nranks, bytes, dtype);
  if (algo == MSCCLPP_AMD_ALGO_FULLMESH || algo == MSCCLPP_AMD_ALGO_RSAG) {
    return bulkScratchRequired(nranks, bytes, (size_t)1 << 40, nullptr, 64);
  }
  if (algo == MSCCLPP_AMD_ALGO_TEST_K6 || algo == MSCCLPP_AMD_ALGO_TEST_K7) return testLLScratchRequired(nranks, bytes);
  if (algo == MSCCLPP_AMD_ALGO_TEST_K2) return testK2ScratchRequired(nranks, bytes);
  if (algo == MSCCLPP_AMD_ALGO_RSAG_ZC || algo == MSCCLPP_AMD_ALGO_TEST_K5) return 0;  // peers' buffers read in place
  if (algo == MSCCLPP_AMD_ALGO_RSAG_PIPELINE) return mscclppAmdScratchRequiredShape(algo, nranks, bytes, dtype, 0, 0);
  return 0;
}

// As above for an explicit launch shape (nblocks / nthreads <= 0: the algorithm's defaults).  Only
// the pipelined RS+AG depends on the shape: it needs at least one stage of 2 * n * (R * T * 4) 16-byte
// units, R = nblocks reduce workgroups of T = nthreads lanes; more stages deepen the pipeline.
size_t mscclppAmdScratchRequiredShape(int algo, int nranks, size_t bytes, int dtype, int nblocks, int nthreads) {
  if (algo != MSCCLPP_AMD_ALGO_RSAG_PIPELINE) return mscclppAmdScratchRequired(algo, nranks, bytes, dtype);
  if (nblocks <= 0) nblocks = 32;
  if (nthreads <= 0) nthreads = 512;
  return 2 * (size_t)nranks * (size_t)nblocks * (size_t)nthreads * 4 * 16;
}

// The tuned-config store (tuning.cpp): the built-in table is algorithm_selector.cc:91-139 for an
// AMD node (<= 16 KiB one-hop LL8, <= 1 MiB two-hop LL16, larger buckets the bulk all-pairs path);
// MSCCLPP_AMD_TUNED_CONFIG / mscclppAmdTunedConfigLoad profiles for this SKU and rank count come first.
int mscclppAmdSelectAlgo(int nranks, size_t bytes, int dtype) {
  (void)dtype;
  std::string name;
  int nb = 0, nt = 0;
  try {
    if (tunedConfig("allreduce", nranks, bytes, name, nb, nt)) {
      const int code = algoCodeOf(name);
      if (code > 0) return code;
    }
  } catch (...) {
  }
  if (bytes <= ((size_t)1 << 14)) return MSCCLPP_AMD_ALGO_ALLPAIR;
  if (bytes <= ((size_t)1 << 20)) return MSCCLPP_AMD_ALGO_PACKET;
  return MSCCLPP_AMD_ALGO_FULLMESH;
}

// =============================================================================================
// NCCL ABI (nccl.cc)
// =============================================================================================
ncclResult_t ncclGetVersion(int* version) {
  if (!version) return ncclInvalidArgument;
  *version = NCCL_VERSION_CODE;
  return ncclSuccess;
}

ncclResult_t ncclGetUniqueId(ncclUniqueId* uniqueId) {
  return (ncclResult_t)guarded([&] {
    if (!uniqueId) return (int)ncclInvalidArgument;
    BootstrapId id = bootstrapCreateRoot();
    std::memcpy(uniqueId, &id, sizeof(id));
    return (int)ncclSuccess;
  });
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId commId, int rank) {
  return (ncclResult_t)host::commInitRank(comm, nranks, &commId, rank, 0);
}

}  // extern "C"

namespace mscclpp_amd {
namespace host {
int commInitRank(ncclComm_t* comm, int nranks, const void* commId, int rank, int timeoutSec) {
  if (timeoutSec <= 0) {  // every caller without a timeout of its own: the environment's, else 600 s
    const char* to = std::getenv("MSCCLPP_AMD_BOOTSTRAP_TIMEOUT_S");
    timeoutSec = to && std::atoi(to) > 0 ? std::atoi(to) : 600;
  }
  return guarded([&] {
    if (!comm || !commId) return (int)ncclInvalidArgument;
    if (nranks <= 0 || rank < 0 || rank >= nranks) return (int)ncclInvalidArgument;
    if (nranks > MSCCLPP_AMD_MAX_RANKS) {
      warn("mscclpp_amd covers one MI355X node: at most 8 ranks");
      return (int)ncclInvalidUsage;
    }
    BootstrapId id;
    std::memcpy(&id, commId, sizeof(id));
    if (!bootstrapIdValid(id)) return (int)ncclInvalidArgument;
    auto c = std::make_unique<ncclComm>();
    c->rank = rank;
    c->nranks = nranks;
    HIPCHECK(hipGetDevice(&c->device));
    info("rank " + std::to_string(rank) + ": bootstrap connect");
    c->boot = std::make_unique<StarBootstrap>(rank, nranks, id, timeoutSec > 0 ? timeoutSec : 600);
    info("rank " + std::to_string(rank) + ": bootstrap connected");
    const size_t tokBytes = sizeof(uint64_t) * MSCCLPP_AMD_MAX_RANKS * MSCCLPP_AMD_MAX_CHANNELS;
    c->tokens = (uint64_t*)allocUncached(tokBytes);
    HIPCHECK(hipMalloc((void**)&c->expected, tokBytes));
    memsetSync(c->expected, 0, tokBytes);
    HIPCHECK(hipMalloc((void**)&c->flags, MSCCLPP_AMD_FLAG_SLOTS * sizeof(uint32_t)));
    {
      std::vector<uint32_t> ones(MSCCLPP_AMD_FLAG_SLOTS, 1u);
      HIPCHECK(hipMemcpy(c->flags, ones.data(), ones.size() * 4, hipMemcpyHostToDevice));
    }
    HIPCHECK(hipMalloc((void**)&c->err, 256));
    memsetSync(c->err, 0, 256);
    if (nranks > 1) {
      info("rank " + std::to_string(rank) + ": exchanging semaphore tokens");
      c->peerTok = c->exchange(c->tokens);
      info("rank " + std::to_string(rank) + ": tokens mapped; allocating LL scratch");
      for (int r = 0; r < nranks; ++r) c->peerTokens[r] = (uint64_t*)c->peerTok[r];
      c->ensure(c->llScratch, c->llBytes, c->peerLL, (size_t)64 << 20);
      // The bulk scratch at its final size now (the reference allocates its scratch once at init
      // too, nccl.cc:180, :299): every bulk algorithm fits its need into 1 GiB (more passes or
      // fewer pipeline stages beyond), so it is never re-allocated -- and never re-exported -- while
      // the communicator runs.  Re-exporting a fresh allocation mid-run through hipIpcGetMemHandle
      // misbehaved here (8 processes on one GPU): an import that mapped the previous allocation,
      // or `invalid argument` from the export itself (tools/multi_rank_check.py).
      c->ensure(c->bulkScratch, c->bulkBytes, c->peerBulk, bulkScratchInitBytes());
    }
    c->buildAlgorithms();
    initFallbackComm(c.get());  // vendor communicator for operations outside this path (nccl.cc:323-346)
    HIPCHECK(hipDeviceSynchronize());
    c->boot->barrier();
    *comm = c.release();
    return (int)ncclSuccess;
  });
}
}  // namespace host
}  // namespace mscclpp_amd

extern "C" {

ncclResult_t ncclCommInitRankConfig(ncclComm_t* comm, int nranks, ncclUniqueId commId, int rank, ncclConfig_t*) {
  return ncclCommInitRank(comm, nranks, commId, rank);
}

ncclResult_t ncclCommInitAll(ncclComm_t* comm, int ndev, const int*) {
  if (ndev == 1) {
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) return r;
    return ncclCommInitRank(comm, 1, id, 0);
  }
  warn("ncclCommInitAll with more than one device is unavailable (one process per GPU), as in nccl.cc:351-360");
  return ncclInternalError;
}

ncclResult_t ncclCommFinalize(ncclComm_t comm) {
  if (!comm) return ncclInvalidArgument;
  if (comm->fallback && vendorNccl()->CommFinalize) {  // nccl.cc:367-373
    const ncclResult_t r = vendorNccl()->CommFinalize((ncclComm_t)comm->fallback);
    if (r != ncclSuccess) return r;
  }
  return ncclSuccess;
}

// The communicator is deleted whatever the teardown reports: a failed step is returned as the
// result, never left behind as a half-destroyed handle.
ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  if (!comm) return ncclInvalidArgument;
  const int a = guarded([&] {
    destroyFallbackComm(comm, false);
    return (int)ncclSuccess;
  });
  const int b = guarded([&] {
    comm->destroy();
    return (int)ncclSuccess;
  });
  delete comm;
  return (ncclResult_t)(a != ncclSuccess ? a : b);
}

ncclResult_t ncclCommAbort(ncclComm_t comm) {
  if (!comm) return ncclSuccess;
  const int a = guarded([&] {
    destroyFallbackComm(comm, true);
    return (int)ncclSuccess;
  });
  const int b = guarded([&] {
    comm->destroy();
    return (int)ncclSuccess;
  });
  delete comm;
  return (ncclResult_t)(a != ncclSuccess ? a : b);
}

const char* ncclGetErrorString(ncclResult_t result) {
  switch (result) {
    case ncclSuccess: return "no error";
    case ncclUnhandledCudaError: return "unhandled HIP error";
    case ncclSystemError: return "unhandled system error";
    case ncclInternalError: return "internal error";
    case ncclInvalidArgument: return "invalid argument";
    case ncclInvalidUsage: return "invalid usage";
    case ncclRemoteError: return "remote process exited or there was a network error";
    case ncclInProgress: return "NCCL operation in progress";
    default: return "unknown result code";
  }
}

const char* ncclGetLastError(ncclComm_t) { return gLastError.c_str(); }

ncclResult_t ncclCommGetAsyncError(ncclComm_t comm, ncclResult_t* asyncError) {
  if (!comm || !asyncError) return ncclInvalidArgument;
  // Polled by frameworks' watchdog threads: read the error word on a stream of its own, never the
  // null stream (which would wait behind every blocking stream's queued collectives).
  uint32_t code = 0;
  if (!comm->errStream && hipStreamCreateWithFlags(&comm->errStream, hipStreamNonBlocking) != hipSuccess) {
    *asyncError = ncclUnhandledCudaError;
    return ncclSuccess;
  }
  if (hipMemcpyAsync(&code, comm->err, sizeof(code), hipMemcpyDeviceToHost, comm->errStream) != hipSuccess ||
      hipStreamSynchronize(comm->errStream) != hipSuccess) {
    *asyncError = ncclUnhandledCudaError;
    return ncclSuccess;
  }
  *asyncError = code ? ncclRemoteError : ncclSuccess;
  return ncclSuccess;
}

ncclResult_t ncclCommCount(const ncclComm_t comm, int* count) {
  if (!comm || !count) return ncclInvalidArgument;
  *count = comm->nranks;
  return ncclSuccess;
}

ncclResult_t ncclCommCuDevice(const ncclComm_t comm, int* device) {
  if (!comm || !device) return ncclInvalidArgument;
  *device = comm->device;
  return ncclSuccess;
}

ncclResult_t ncclCommUserRank(const ncclComm_t comm, int* rank) {
  if (!comm || !rank) return ncclInvalidArgument;
  *rank = comm->rank;
  return ncclSuccess;
}

// Select through the communicator's AlgorithmCollection and execute (nccl.cc:578-596): the user's
// selector first, the built-in one as fallback; no algorithm -> ncclInvalidUsage (there is no
// NCCL/RCCL underneath to fall back to).
static int selectAndExecute(ncclComm_t comm, const char* collective, const void* sendbuff, void* recvbuff,
                            size_t messageSize, size_t inBytes, size_t outBytes, ncclDataType_t datatype,
                            ncclRedOp_t op, void* stream) {
  using namespace mscclpp_amd;
  static const std::unordered_map<std::string, std::vector<uint64_t>> kNoHints;
  const DataType dtype = dataTypeFromNccl(datatype);
  // With only the built-in selector the choice is a function of (collective, size, dtype) and the
  // tuned store: memoise it, and the tuned shape with it (one store lookup per new key instead of
  // two per call).  `collective` is one of this file's literals, so its address names it.
  const bool memoOk = !comm->algos->hasAlgorithmSelector();
  std::shared_ptr<Algorithm> algo;
  int nb = 0, nt = 0;
  if (memoOk) {
    const uint64_t gen = tunedGeneration();
    const size_t h = (messageSize * 0x9E3779B97F4A7C15ull) ^ ((size_t)collective >> 3) ^ (size_t)datatype;
    std::lock_guard<std::mutex> lk(comm->selMu);
    ncclComm::SelMemo& m = comm->selMemo[(h >> 7) % comm->selMemo.size()];
    if (m.coll == collective && m.size == messageSize && m.dtype == (int)datatype && m.gen == gen && m.algo) {
      algo = m.algo;
      nb = m.nb;
      nt = m.nt;
    } else {
      CollectiveRequest req{comm->nranks, comm->nranks, comm->rank, sendbuff, recvbuff, messageSize,
                            (hipStream_t)stream, std::string(collective), dtype, kNoHints};
      algo = comm->algos->selectAlgorithm(req);
      if (algo) {
        const auto& tags = algo->tags();
        if (tags.find("default") != tags.end()) {  // a built-in: its tuned shape, resolved once here
          std::string name;
          int tb = 0, tt = 0;
          if (tunedConfig(collective, comm->nranks, messageSize, name, tb, tt) && name == algo->name()) {
            nb = tb;
            nt = tt;
          }
          if (nb <= 0 && nt <= 0) {
            nb = kTunedShapeResolved;
            nt = 0;
          }
        }
        m = ncclComm::SelMemo{collective, messageSize, (int)datatype, gen, algo, nb, nt};
      }
    }
  } else {
    CollectiveRequest req{comm->nranks, comm->nranks, comm->rank, sendbuff, recvbuff, messageSize,
                          (hipStream_t)stream, std::string(collective), dtype, kNoHints};
    algo = comm->algos->selectAlgorithm(req);
  }
  if (!algo) {
    warn(std::string("no algorithm selected for ") + collective + " of " + std::to_string(messageSize) + " bytes");
    return ncclInvalidUsage;
  }
  if (algo->type() == AlgorithmType::DSL && !comm->executor) comm->executor = std::make_shared<Executor>(comm->cxx);
  const ReduceOp rop = op == ncclSum ? SUM : op == ncclMin ? MIN : NOP;
  const int rc = (int)algo->execute(comm->cxx, sendbuff, recvbuff, inBytes, outBytes, dtype, rop, (hipStream_t)stream,
                                    comm->executor, nb, nt);
  if (rc != ncclSuccess)
    warn(std::string(collective) + " via " + algo->name() + " of " + std::to_string(messageSize) +
         " bytes failed with code " + std::to_string(rc) + " (HIP: " + hipGetErrorString(hipPeekAtLastError()) + ")");
  return rc;
}

ncclResult_t ncclAllReduce(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype,
                           ncclRedOp_t op, ncclComm_t comm, void* stream) {
  return (ncclResult_t)guarded([&] {
    if (!comm) return (int)ncclInvalidArgument;
    const size_t tb = ncclTypeBytes(datatype);
    const size_t bytes = count * tb;
    if (comm->nranks == 1) {  // nccl.cc:610-615
      if (sendbuff != recvbuff && bytes)
        HIPCHECK(hipMemcpyAsync(recvbuff, sendbuff, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
      return (int)ncclSuccess;
    }
    if (!sendbuff || !recvbuff || count == 0 || tb == 0) return (int)ncclInvalidArgument;  // nccl.cc:617-622
    const int dt = dtypeFromNccl(datatype);
    const int o = opFromNccl(op);
    if (comm->fallback && (dt < 0 || o < 0 || forcedFallback("allreduce")))  // nccl.cc:628-632
      return (int)vendorNccl()->AllReduce(sendbuff, recvbuff, count, datatype, op, (ncclComm_t)comm->fallback, stream);
    if (dt < 0 || o < 0) {
      warn("unsupported dtype/op for AllReduce (supported: fp16, bf16, fp32, int32, uint32, uint8, fp8 e4m3/e5m2 x sum, min)");
      return (int)ncclInvalidArgument;
    }
    return selectAndExecute(comm, "allreduce", sendbuff, recvbuff, bytes, bytes, bytes, datatype, op, stream);
  });
}

ncclResult_t ncclReduceScatter(const void* sendbuff, void* recvbuff, size_t recvcount, ncclDataType_t datatype,
                               ncclRedOp_t op, ncclComm_t comm, void* stream) {
  return (ncclResult_t)guarded([&] {
    if (!comm) return (int)ncclInvalidArgument;
    const size_t tb = ncclTypeBytes(datatype);
    const size_t bytes = recvcount * tb;
    if (comm->nranks == 1) {  // nccl.cc:662-672
      if (sendbuff != recvbuff && bytes)
        HIPCHECK(hipMemcpyAsync(recvbuff, sendbuff, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
      return (int)ncclSuccess;
    }
    if (!sendbuff || !recvbuff || recvcount == 0 || tb == 0) return (int)ncclInvalidArgument;
    const int dt = dtypeFromNccl(datatype), o = opFromNccl(op);
    if (comm->fallback && (dt < 0 || o < 0 || forcedFallback("reducescatter")))  // nccl.cc:682-686
      return (int)vendorNccl()->ReduceScatter(sendbuff, recvbuff, recvcount, datatype, op, (ncclComm_t)comm->fallback,
                                              stream);
    if (dt < 0 || o < 0) return (int)ncclInvalidArgument;
    const size_t total = bytes * (size_t)comm->nranks;  // messageSize = bytes * nRank (nccl.cc:692-697)
    return selectAndExecute(comm, "reducescatter", sendbuff, recvbuff, total, total, bytes, datatype, op, stream);
  });
}

ncclResult_t ncclAllGather(const void* sendbuff, void* recvbuff, size_t sendcount, ncclDataType_t datatype,
                           ncclComm_t comm, void* stream) {
  return (ncclResult_t)guarded([&] {
    if (!comm) return (int)ncclInvalidArgument;
    const size_t tb = ncclTypeBytes(datatype);
    const size_t bytes = sendcount * tb;
    if (comm->nranks == 1) {
      if (sendbuff != recvbuff && bytes)
        HIPCHECK(hipMemcpyAsync(recvbuff, sendbuff, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
      return (int)ncclSuccess;
    }
    if (!sendbuff || !recvbuff || sendcount == 0 || tb == 0) return (int)ncclInvalidArgument;
    if (comm->fallback && (bytes % 16 || forcedFallback("allgather")))  // nccl.cc:736-739
      return (int)vendorNccl()->AllGather(sendbuff, recvbuff, sendcount, datatype, (ncclComm_t)comm->fallback, stream);
    if (tb != 2 && tb != 4 && tb != 1 && tb != 8) return (int)ncclInvalidArgument;
    return selectAndExecute(comm, "allgather", sendbuff, recvbuff, bytes, bytes, bytes * (size_t)comm->nranks,
                            datatype, ncclSum, stream);
  });
}

// Native operations run when called (a group does not defer them); with a vendor library the group
// calls are forwarded so grouped vendor operations (send/recv) keep their semantics (nccl.cc:823-838).
ncclResult_t ncclGroupStart(void) { return vendorNccl() ? vendorNccl()->GroupStart() : ncclSuccess; }
ncclResult_t ncclGroupEnd(void) { return vendorNccl() ? vendorNccl()->GroupEnd() : ncclSuccess; }

ncclResult_t ncclMemAlloc(void** ptr, size_t size) {
  return (ncclResult_t)guarded([&] {
    if (!ptr || !size) return (int)ncclInvalidArgument;
    HIPCHECK(hipMalloc(ptr, size));
    return (int)ncclSuccess;
  });
}

ncclResult_t ncclMemFree(void* ptr) {
  return (ncclResult_t)guarded([&] {
    if (ptr) HIPCHECK(hipFree(ptr));
    return (int)ncclSuccess;
  });
}

// =============================================================================================
// communicator extensions
// =============================================================================================
int mscclppAmdCommAllReduce(ncclComm_t comm, const void* sendbuff, void* recvbuff, size_t count, int ncclDtype,
                            int ncclOp, int algo, int nblocks, int nthreads, void* stream) {
  return mscclppAmdCommAllReduceAccum(comm, sendbuff, recvbuff, count, ncclDtype, ncclOp, -1, algo, nblocks, nthreads,
                                      stream);
}

int mscclppAmdReduceType(int ncclDtype, int accumNcclDtype) { return reduceTypeFromNccl(ncclDtype, accumNcclDtype); }

int mscclppAmdCommAllReduceAccum(ncclComm_t comm, const void* sendbuff, void* recvbuff, size_t count, int ncclDtype,
                                 int ncclOp, int accumNcclDtype, int algo, int nblocks, int nthreads, void* stream) {
  return guarded([&] {
    const size_t tb = ncclTypeBytes((ncclDataType_t)ncclDtype);
    if (comm && comm->nranks == 1) {  // a copy, before any argument check (nccl.cc:610-615)
      if (sendbuff != recvbuff && count * tb)
        HIPCHECK(hipMemcpyAsync(recvbuff, sendbuff, count * tb, hipMemcpyDeviceToDevice, (hipStream_t)stream));
      return (int)ncclSuccess;
    }
    if (!comm || !sendbuff || !recvbuff || count == 0) return (int)ncclInvalidArgument;
    const int dt = reduceTypeFromNccl(ncclDtype, accumNcclDtype);
    const int o = opFromNccl((ncclRedOp_t)ncclOp);
    if (dt < 0 || o < 0 || tb == 0) return (int)ncclInvalidArgument;
    return comm->allReduce(sendbuff, recvbuff, count * tb, dt, o, algo, nblocks, nthreads, (hipStream_t)stream);
  });
}

int mscclppAmdCommBarrier(ncclComm_t comm) {
  return guarded([&] {
    if (!comm) return (int)ncclInvalidArgument;
    comm->boot->barrier();
    return (int)ncclSuccess;
  });
}

int mscclppAmdCommGetDeviceError(ncclComm_t comm, uint32_t* code, int clear) {
  return guarded([&] {
    if (!comm || !code) return (int)ncclInvalidArgument;
    HIPCHECK(hipMemcpy(code, comm->err, sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (clear) memsetSync(comm->err, 0, sizeof(uint32_t));
    return (int)ncclSuccess;
  });
}

int mscclppAmdCommGetDeviceErrorDetail(ncclComm_t comm, uint32_t* words4, int clear) {
  return guarded([&] {
    if (!comm || !words4) return (int)ncclInvalidArgument;
    HIPCHECK(hipMemcpy(words4, comm->err, 4 * sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (clear) memsetSync(comm->err, 0, 4 * sizeof(uint32_t));
    return (int)ncclSuccess;
  });
}

int mscclppAmdCommRegistrationStats(ncclComm_t comm, size_t* userRegistrations, size_t* liveMappings,
                                    size_t* retiredMappings) {
  if (!comm) return ncclInvalidArgument;
  std::lock_guard<std::mutex> lk(comm->mu);
  if (userRegistrations) *userRegistrations = comm->userRegs.size();
  if (liveMappings) *liveMappings = liveIpcMappings();
  if (retiredMappings) {  // mappings still waiting for their last launches to complete
    comm->flushRetired();
    size_t k = 0;
    for (const auto& r : comm->retired) k += r.maps.size();
    *retiredMappings = k;
  }
  return ncclSuccess;
}

int mscclppAmdCommRegistrationExchanges(ncclComm_t comm, uint64_t* allocationExchanges, uint64_t* offsetExchanges,
                                        int* symmetricMemory) {
  if (!comm) return ncclInvalidArgument;
  std::lock_guard<std::mutex> lk(comm->mu);
  if (allocationExchanges) *allocationExchanges = comm->allocExchanges;
  if (offsetExchanges) *offsetExchanges = comm->offsetExchanges;
  if (symmetricMemory) *symmetricMemory = comm->symmetricMemory ? 1 : 0;
  return ncclSuccess;
}

int mscclppAmdCommScratch(ncclComm_t comm, void** scratch, size_t* bytes) {
  if (!comm || !scratch || !bytes) return ncclInvalidArgument;
  *scratch = comm->llScratch;
  *bytes = comm->llBytes;
  return ncclSuccess;
}

int mscclppAmdCommFlags(ncclComm_t comm, uint32_t** flags) {
  if (!comm || !flags) return ncclInvalidArgument;
  *flags = comm->flags;
  return ncclSuccess;
}

int mscclppAmdCommAllGatherHost(ncclComm_t comm, const void* sendbuf, void* recvbuf, size_t bytes) {
  return guarded([&] {
    if (!comm) return (int)ncclInvalidArgument;
    comm->boot->allGather(sendbuf, recvbuf, bytes);
    return (int)ncclSuccess;
  });
}

// ---- bootstrap (setup plane only; host code, usable without a GPU) -------------------------
int mscclppAmdBootstrapCreate(int rank, int nranks, const void* uniqueId, void** handle) {
  return guarded([&] {
    if (!uniqueId || !handle || nranks <= 0 || rank < 0 || rank >= nranks) return (int)ncclInvalidArgument;
    BootstrapId id;
    std::memcpy(&id, uniqueId, sizeof(id));
    if (!bootstrapIdValid(id)) return (int)ncclInvalidArgument;
    *handle = new StarBootstrap(rank, nranks, id, 120);
    return (int)ncclSuccess;
  });
}

int mscclppAmdBootstrapAllGather(void* handle, const void* sendbuf, void* recvbuf, size_t bytes) {
  return guarded([&] {
    if (!handle) return (int)ncclInvalidArgument;
    static_cast<StarBootstrap*>(handle)->allGather(sendbuf, recvbuf, bytes);
    return (int)ncclSuccess;
  });
}

int mscclppAmdBootstrapBarrier(void* handle) {
  return guarded([&] {
    if (!handle) return (int)ncclInvalidArgument;
    static_cast<StarBootstrap*>(handle)->barrier();
    return (int)ncclSuccess;
  });
}

int mscclppAmdBootstrapDestroy(void* handle) {
  delete static_cast<StarBootstrap*>(handle);
  return ncclSuccess;
}

}  // extern "C"
