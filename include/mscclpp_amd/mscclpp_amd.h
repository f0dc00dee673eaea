/*
 * mscclpp_amd extension C ABI (libmscclpp_amd.so).  Plain pointers and sizes only.
 *
 * The NCCL drop-in entry points live in nccl.h.  This header adds what the reference exposes
 * through its C++ API (include/mscclpp/core.hpp, algorithm.hpp, gpu_utils.hpp) and that the
 * parity tests and the benchmark need:
 *   - uncached device allocation and flag buffers (gpu_utils.cc:139-147, algorithm.cc:251-268)
 *   - the 1-GPU LL16 pack+sum+unpack microbench kernel (BASELINE config 2)
 *   - explicit-view AllReduce launchers: every rank's buffers and mapped peer pointers are passed
 *     in, so the same kernels run either one rank per process (views = 1) or several ranks of a
 *     single process on one GPU (views = n, "in-process ranks", used by the parity tests)
 *   - Algorithm::execute with an explicit algorithm (algorithm.hpp:108-113)
 *
 * Return codes are ncclResult_t values (0 = success, 1 = HIP error, 3 = internal, 4 = invalid
 * argument, 5 = invalid usage).
 */
#ifndef MSCCLPP_AMD_H_
#define MSCCLPP_AMD_H_

#include <stddef.h>
#include <stdint.h>

#include "nccl.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MSCCLPP_AMD_MAX_RANKS 8
#define MSCCLPP_AMD_FLAG_SLOTS 4096
#define MSCCLPP_AMD_MAX_CHANNELS 256

/* dtype / op codes of the extension API (ncclDataType_t / ncclRedOp_t are mapped onto these) */
enum { MSCCLPP_AMD_F16 = 0, MSCCLPP_AMD_BF16 = 1, MSCCLPP_AMD_F32 = 2, MSCCLPP_AMD_I32 = 3, MSCCLPP_AMD_U32 = 4 };
/* OCP FP8 (gfx950 hardware formats; the reference's DataType::FLOAT8_E4M3FN / FLOAT8_E5M2,
 * gpu_data_types.hpp:170-183).  The code also names the accumulation type of
 * Algorithm::execute(..., accumDtype) (algorithm.hpp:108-113, common.hpp:89-100): the element
 * type itself (AUTO), half or float. */
enum {
  MSCCLPP_AMD_E4M3 = 5,
  MSCCLPP_AMD_E5M2 = 6,
  MSCCLPP_AMD_E4M3_ACC_F16 = 7,
  MSCCLPP_AMD_E5M2_ACC_F16 = 8,
  MSCCLPP_AMD_E4M3_ACC_F32 = 9,
  MSCCLPP_AMD_E5M2_ACC_F32 = 10,
  /* uint8 (ncclUint8; Adapter<Op, uint8_t, uint8_t>, common.hpp:132-133): wrapping add / unsigned
   * min per byte (gpu_data_types.hpp:577-640) */
  MSCCLPP_AMD_U8 = 11,
  /* the software float8 e4m3b15 (DataType::FLOAT8_E4M3B15, gpu_data_types.hpp:78-155; no NCCL
   * dtype): accumulated in itself, half or float, as the OCP codes above */
  MSCCLPP_AMD_E4M3B15 = 12,
  MSCCLPP_AMD_E4M3B15_ACC_F16 = 13,
  MSCCLPP_AMD_E4M3B15_ACC_F32 = 14,
  MSCCLPP_AMD_NUM_DTYPES = 15
};
enum { MSCCLPP_AMD_SUM = 0, MSCCLPP_AMD_MIN = 1 };

/* AllReduce algorithms (names follow the reference's AlgorithmCollection keys) */
enum {
  MSCCLPP_AMD_ALGO_AUTO = 0,
  MSCCLPP_AMD_ALGO_PACKET = 1,   /* default_allreduce_packet: LL16 two-hop (allreduce_packet.cu:15-151) */
  MSCCLPP_AMD_ALGO_ALLPAIR = 2,  /* default_allreduce_allpair_packet: LL8 one-hop (allreduce_allpair_packet.cu:15-69) */
  MSCCLPP_AMD_ALGO_FULLMESH = 3, /* default_allreduce_fullmesh: bulk all-pairs RS+AG (allreduce_fullmesh.cu:24-166) */
  MSCCLPP_AMD_ALGO_RSAG = 4,     /* default_allreduce_rsag: ring-order bulk RS+AG (allreduce_rsag.cu:33-128) */
  MSCCLPP_AMD_ALGO_RSAG_ZC = 5,  /* default_allreduce_rsag_zero_copy: reads peers' inputs, writes peers' outputs,
                                    no scratch (allreduce_rsag_zero_copy.cu:41-112) */
  MSCCLPP_AMD_ALGO_RSAG_PIPELINE = 6, /* default_allreduce_rsag_pipeline: put / reduce / recv workgroups
                                         pipelined over a circular scratch (allreduce_rsag_pipeline.cu:85-222) */
  /* the int32 kernels of the mscclpp-test harness (test/mscclpp-test/allreduce_test.cu), by number */
  MSCCLPP_AMD_ALGO_TEST_K2 = 102, /* allreduce2, one node: LL16 one-hop all-pairs, harness scratch layout (:841-943) */
  MSCCLPP_AMD_ALGO_TEST_K5 = 105, /* allreduce5 (AMD branch): in-place RS by remote reads + ring AG by gets (:959-970) */
  MSCCLPP_AMD_ALGO_TEST_K6 = 106, /* allreduce6: LL16 two-hop, harness scratch layout (:972-1034) */
  MSCCLPP_AMD_ALGO_TEST_K7 = 107  /* allreduce7: LL8 two-hop, harness scratch layout (:1036-1093) */
};

/* One rank's view of the buffers of an AllReduce.  Pointers to other ranks' memory are the
 * addresses at which this rank has them mapped (IPC), or plain device pointers for in-process
 * ranks.  Entry [rank] of every peer array is this rank's own buffer. */
typedef struct {
  const void* input;
  void* output;
  void* scratch;                                   /* own scratch (two halves) */
  void* peerScratch[MSCCLPP_AMD_MAX_RANKS];        /* rank q's scratch as mapped here */
  void* peerOutput[MSCCLPP_AMD_MAX_RANKS];         /* rank q's output (bulk direct writes) */
  uint64_t* tokens;                                /* own inbound tokens [MAX_RANKS][MAX_CHANNELS] */
  uint64_t* peerTokens[MSCCLPP_AMD_MAX_RANKS];     /* rank q's tokens as mapped here */
  uint64_t* expected;                              /* own expected counters [MAX_RANKS][MAX_CHANNELS] */
  uint32_t* flags;                                 /* MSCCLPP_AMD_FLAG_SLOTS words, initialised to 1,
                                                      16-byte aligned */
  uint32_t* err;                                   /* device error word (0 = ok) */
  uint64_t scratchBytes;
  int32_t rank;
  int32_t pad;
  const void* peerInput[MSCCLPP_AMD_MAX_RANKS];    /* rank q's input as mapped here (zero-copy reads) */
  uint64_t* pipeSems;                              /* rsag_pipeline: 3 x 256 + 64 intra-launch counters,
                                                      zero before the first launch; every launch leaves
                                                      them zero (graph replays need no memset) */
} mscclppAmdRankView;

/* ---- memory ------------------------------------------------------------------------------- */
/* Uncached memory (hipDeviceMallocUncached, zeroed; the reference's GpuBuffer on AMD,
 * gpu_utils.cc:139-147) comes from a process-lifetime pool: mscclppAmdFree hands a pooled block back
 * to the pool, never to HIP, so no later allocation is placed where uncached memory was (DESIGN.md
 * §21).  The free does not synchronize: the block is reused only after a device synchronize, paid by
 * the allocation that reuses it.  mscclppAmdFree hipFree's anything else.
 * mscclppAmdUncachedPoolStats: bytes allocated from HIP, in use, and free in the pool. */
int mscclppAmdMallocUncached(void** ptr, size_t bytes);
int mscclppAmdMalloc(void** ptr, size_t bytes);
int mscclppAmdFree(void* ptr);
int mscclppAmdUncachedPoolStats(size_t* held, size_t* inUse, size_t* freeBytes);
/* Imports of peers' memory in this process: IPC mappings open now, and how many of them are kept
 * imports of peers' pooled uncached blocks (scratch, tokens, GpuBuffer), which stay mapped until
 * the process exits -- the import-side twin of the pool.  mscclppAmdIpcKeptRanges
 * writes up to `cap` (mapped address, bytes) pairs of the kept imports and their count to *n.  Any
 * pointer may be NULL. */
int mscclppAmdIpcStats(size_t* openMappings, size_t* keptImports);
int mscclppAmdIpcKeptRanges(uint64_t* addrs, uint64_t* bytes, size_t cap, size_t* n);
/* Forget the kept imports (after a device synchronize): each closes unless a live communicator still
 * holds it.  For a long-lived process whose peers come and go (an elastic job re-creating its peer
 * processes): a kept import keeps the exited peer's memory alive.  Call it only with no communicator
 * of the departed peers left, and expect this process's next allocations to be placed where the
 * closed mappings were -- the hazard DESIGN.md §21 describes, which the kept imports otherwise rule
 * out. */
int mscclppAmdIpcReleaseKept(size_t* released);
int mscclppAmdFlagsInit(uint32_t* flags, void* stream);

/* ---- 1-GPU microbench (BASELINE config 2) ------------------------------------------------- */
/* out = x (op) unpack(pack(y, flag)); pkts: 2*bytes of (uncached) device memory; bytes % 16 == 0.
 * 256-lane workgroups with 4 KiB per round; nblocks <= 0 selects the default grid (one workgroup per
 * 4 KiB up to 1024 of them), nblocks > 0 that grid (<= 1024).  budgetTicks: spin budget in 10 ns
 * ticks.  flags: MSCCLPP_AMD_FLAG_SLOTS words, 16-byte aligned.  The packet hand-off runs between the
 * waves of each workgroup. */
int mscclppAmdSelfReduceLL16(const void* x, const void* y, void* pkts, void* out, size_t bytes, int dtype, int op,
                             uint32_t* flags, int nblocks, uint64_t budgetTicks, uint32_t* err, void* stream);
/* The default shape for `bytes`: waves per workgroup, KiB per wave and round, workgroups, skewed. */
int mscclppAmdSelfReduceLL16DefaultShape(size_t bytes, int* waves, int* units, int* nblocks, int* skew);

/* Ceiling helpers used by the benchmark.  mscclppAmdCopy is a plain streaming copy (HBM ceiling);
 * mscclppAmdCopyJobs runs njobs copies in ONE launch, blocksPerJob workgroups each (the xGMI probe:
 * all peers' links driven from one kernel on one stream).  (Kernel shape sweeps and first-poll miss
 * counts of the self-reduce live in the test diagnostics library, tests/bin/libselfreduce_diag.so.) */
int mscclppAmdCopy(const void* src, void* dst, size_t bytes, int nblocks, void* stream);
int mscclppAmdCopyJobs(const void* const* srcs, void* const* dsts, const size_t* bytes, int njobs, int blocksPerJob,
                       void* stream);
/* The same with the cache policy of the loads / stores: 0 = sc0 sc1 (system scope, what the
 * collectives use for remote accesses), 1 = plain, 2 = nt, 3 = sc1 (agent scope).  Combinations
 * carried: any store policy with system loads; plain or system stores with plain loads; system stores
 * with nt or agent loads.  4 = a combination not carried. */
int mscclppAmdCopyJobsPolicy(const void* const* srcs, void* const* dsts, const size_t* bytes, int njobs,
                             int blocksPerJob, int loadPolicy, int storePolicy, void* stream);
/* The self-reduce's exact memory accesses (Y read, packets stored and the partner's read two rounds
 * late, X read, O written: 7 * bytes over the same buffers, grid and rounds) with no flags, readiness
 * tests or LDS: the streaming ceiling of that access mix.  bytes: a multiple of 8 KiB; pkts: 2 * bytes.
 * The output is meaningless. */
int mscclppAmdSelfReduceStream(const void* x, const void* y, void* pkts, void* out, size_t bytes, void* stream);
/* An independent streaming ceiling of the same 4:3 read:write mix, with none of the self-reduce's
 * layout or grid: X, Y (bytes each) and pin (2 * bytes) read, pout (2 * bytes) and out written, one
 * grid-stride loop, 2048 workgroups by default, non-temporal accesses.  bytes % 4096 == 0. */
int mscclppAmdMixStream(const void* x, const void* y, const void* pin, void* pout, void* out, size_t bytes, int nblocks,
                        void* stream);

/* ---- explicit-view AllReduce ------------------------------------------------------------- */
/* Launch `algo` for `nviews` ranks of an `nranks`-rank AllReduce in ONE kernel launch (views[i]
 * is handled by blockIdx.y == i).  nviews == 1 is the one-rank-per-process form; nviews ==
 * nranks runs every rank of the collective inside this process.  Every workgroup waits on other
 * ranks' workgroups, so nblocks * nviews workgroups must be resident at once; a grid that is not
 * returns ncclInvalidUsage (5) without launching. */
int mscclppAmdAllReduceLaunch(int algo, const mscclppAmdRankView* views, int nviews, int nranks, size_t bytes,
                              int dtype, int op, int nblocks, int nthreads, uint64_t budgetTicks, void* stream);
/* coll 0 AllReduce (bytes = buffer), 1 ReduceScatter / 2 AllGather (bytes = nranks * block, block %
 * 16 == 0) through the bulk all-pairs kernel (reduce-scatter / all-gather halves of fullmesh). */
int mscclppAmdCollectiveLaunch(int coll, int algo, const mscclppAmdRankView* views, int nviews, int nranks,
                               size_t bytes, int dtype, int op, int nblocks, int nthreads, uint64_t budgetTicks,
                               void* stream);
/* Scratch bytes per rank (both halves) that `algo` needs for `bytes` (0 if unsupported).  For the
 * pipelined RS+AG this is one stage at the default shape (32 x 512); a larger shape needs
 * mscclppAmdScratchRequiredShape. */
size_t mscclppAmdScratchRequired(int algo, int nranks, size_t bytes, int dtype);
size_t mscclppAmdScratchRequiredShape(int algo, int nranks, size_t bytes, int dtype, int nblocks, int nthreads);
/* Algorithm the selector picks: the tuned-config store's entry for this SKU, rank count and size
 * (built-in table = algorithm_selector.cc:91-139, AMD branch), MSCCLPP_AMD_ALGO_*. */
int mscclppAmdSelectAlgo(int nranks, size_t bytes, int dtype);
/* Tuned-config store (the JSON format of python/mscclpp_benchmark/tuning_config.py): load a file
 * whose profiles take precedence over the built-in table (as MSCCLPP_AMD_TUNED_CONFIG=<path> does at
 * start-up), and query the entry for a collective ("allreduce", "allgather", "reducescatter") of
 * `bytes` on `nranks` ranks: algorithm name and launch shape (0 = default).  Query returns 5 when no
 * entry applies. */
int mscclppAmdTunedConfigLoad(const char* path);
int mscclppAmdTunedConfig(const char* collective, int nranks, size_t bytes, char* algorithm, size_t algorithmLen,
                          int* nblocks, int* nthreads);
/* Where the entry that applies came from: "reference" (the reference's selector restated),
 * "fabric-free" (measured with every rank on one GPU: no link bytes priced), "reference; grid
 * fabric-free", "tuned" (a loaded file's entry without its own "source" tag) or that tag. */
int mscclppAmdTunedConfigSource(const char* collective, int nranks, size_t bytes, char* source, size_t sourceLen);

/* ---- communicator extensions -------------------------------------------------------------- */
// Phase trace of the collective kernels (the reference's NPKit events, npkit.hpp): while a buffer of
// at least MSCCLPP_AMD_TRACE_BYTES device bytes is set, every AllReduce / ReduceScatter / AllGather
// launch of this process has lane 0 of each workgroup write the wall clock (s_memrealtime ticks,
// 100 MHz) at its phase boundaries to buf[(rankView * 256 + workgroup) * 8 + event] (u64).  Events:
// bulk (fullmesh / rsag): 0 start, 1 reduce-scatter puts issued, 2 reduce-scatter handshake done,
// 3 reduce + all-gather stores issued, 4 end; zero-copy: 0 start, 1 entry handshake done, 2 reduce +
// all-gather stores issued, 3 end; LL16: 0 start, 1 step 1 (puts), 2 step 2 (reduce + broadcast),
// 3 step 3 (unpack) done; LL8: 0 start, 1 puts issued, 2 end.  buf = NULL turns it off.  Returns 0,
// or 4 when the buffer is too small.
#define MSCCLPP_AMD_TRACE_BYTES ((size_t)MSCCLPP_AMD_MAX_RANKS * 256 * 8 * 8)
int mscclppAmdTraceSet(void* buf, size_t bytes);

int mscclppAmdCommAllReduce(ncclComm_t comm, const void* sendbuff, void* recvbuff, size_t count, int ncclDtype,
                            int ncclOp, int algo, int nblocks, int nthreads, void* stream);
/* As above with the accumulation type of Algorithm::execute (accumNcclDtype: -1 = AUTO, i.e. the
 * element type; ncclFloat16 / ncclFloat32 for FP8 buffers). */
int mscclppAmdCommAllReduceAccum(ncclComm_t comm, const void* sendbuff, void* recvbuff, size_t count, int ncclDtype,
                                 int ncclOp, int accumNcclDtype, int algo, int nblocks, int nthreads, void* stream);
/* Reduce-type code (MSCCLPP_AMD_*) for an ncclDataType_t and accumulation type (-1 = AUTO), or -1. */
int mscclppAmdReduceType(int ncclDtype, int accumNcclDtype);
int mscclppAmdCommBarrier(ncclComm_t comm);
/* The vendor (RCCL) communicator created beside this one when MSCCLPP_AMD_NCCL_LIB_PATH is set, or
 * NULL (no vendor library, or it refused the communicator). */
int mscclppAmdCommVendorComm(ncclComm_t comm, void** vendorComm);
/* Collective: every rank passes its matching device buffer; peers[r] receives rank r's buffer as
 * mapped in this process (peers[rank] = ptr), MSCCLPP_AMD_MAX_RANKS entries (Communicator::
 * registerMemory of algorithm.hpp; registerMemory + sendMemory/recvMemory in the reference). */
int mscclppAmdCommRegisterBuffer(ncclComm_t comm, void* ptr, void** peers);
/* Collective: close every cached mapping of peers' user buffers (scratch / semaphores stay); call it
 * when buffers that were used with the communicator are freed. */
int mscclppAmdCommDeregisterAll(ncclComm_t comm);
int mscclppAmdCommGetDeviceError(ncclComm_t comm, uint32_t* code, int clear);
/* The communicator's whole error record: words4[0] = the code (as above), words4[1..3] = the detail
 * its first reporter wrote.  kErrPacketTimeout (1): the flag waited for, the byte offset of the
 * packet (or 32-byte unit) in the polled region, the flag word last read there; semaphore timeouts
 * of the bulk and executor kernels: channel / block / expected value.  clear != 0
 * zeroes all four words. */
int mscclppAmdCommGetDeviceErrorDetail(ncclComm_t comm, uint32_t* words4, int clear);
/* Registration cache state: user buffers registered (at most 64, least recently used retired
 * beyond), IPC mappings open in this process (all communicators), mappings waiting for a device
 * synchronize before they close.  Any pointer may be NULL. */
int mscclppAmdCommRegistrationStats(ncclComm_t comm, size_t* userRegistrations, size_t* liveMappings,
                                    size_t* retiredMappings);
/* Host all-gathers made by user-buffer registration so far: one per newly registered allocation,
 * one per new buffer offset inside a registered allocation (none when the communicator runs with
 * MSCCLPP_NCCL_SYMMETRIC_MEMORY, env.hpp:101-107, which *symmetricMemory reports). */
int mscclppAmdCommRegistrationExchanges(ncclComm_t comm, uint64_t* allocationExchanges, uint64_t* offsetExchanges,
                                        int* symmetricMemory);
int mscclppAmdCommScratch(ncclComm_t comm, void** scratch, size_t* bytes);
int mscclppAmdCommFlags(ncclComm_t comm, uint32_t** flags);
/* Bootstrap all-gather of `bytes` per rank (host memory), for harnesses. */
int mscclppAmdCommAllGatherHost(ncclComm_t comm, const void* sendbuf, void* recvbuf, size_t bytes);

/* ---- host-proxy path (PortChannel / FIFO / proxy thread) ------------------------------------
 * Config-1 harness: test/allgather_test_host_offloading.cu on this library.  out[0] = us per
 * kernel (no graph), out[1] = us per kernel (graph of graphIters x 2 kernels), out[2] = 1 if the
 * gathered data is correct, out[3] = NUMA node the proxy thread was bound to (-1 if none). */
int mscclppAmdHostOffloadAllGather(ncclComm_t comm, size_t dataSize, int iters, int graphIters, double* out);
/* PortChannel all-to-all through the proxy (mode 0: put+signal, 1: putWithSignal,
 * 2: putWithSignalAndFlush).  out[0] = us per iteration (wall clock over `iters` back-to-back
 * launches after one untimed launch), out[1] = 1 if correct, out[2] = NUMA node. */
int mscclppAmdPortChannelAllToAll(ncclComm_t comm, size_t chunk, int mode, int iters, double* out);
/* The same with each iteration's own duration (a HIP event before every launch): with outLen >= 7,
 * out[3] = median, out[4] = min, out[5] = max us per iteration, out[6] = index of the slowest one;
 * with outLen >= 8, out[7] = the proxy thread's longest gap between FIFO polls in us over the timed
 * iterations (measured with MSCCLPP_AMD_PROXY_GAP_STATS=1, else 0).  With outLen >= 16 the proxy
 * stamps every timed trigger (ProxyService::enableStamps) and out[8..15] = medians over iterations,
 * us: launch -> this rank's last data copy complete, launch -> its last token update complete, that
 * token update -> kernel end (the wait for the peers' tokens), host submit time of a data copy, of a
 * token update, of a whole trigger; the slowest iteration's launch -> token complete; stamps taken. */
int mscclppAmdPortChannelAllToAllStats(ncclComm_t comm, size_t chunk, int mode, int iters, double* out, int outLen);
/* mscclpp-test allreduce1 (test/mscclpp-test/allreduce_test.cu:730-839): int32 ring RS + AG whose data
 * moves through PortChannels and the host proxy (hipMemcpyAsync).  out[0] = us per AllReduce (graph of
 * `iters` kernels replayed `graphLaunches` times), out[1] = 1 if every element is n(n-1)/2, out[2] =
 * NUMA node of the proxy thread.  nblocks <= 0: the harness's 24 (x 1024 threads). */
int mscclppAmdProxyRingAllReduce(ncclComm_t comm, size_t nelems, int iters, int graphLaunches, int nblocks,
                                 double* out);
int mscclppAmdLaunchRingProxyAllReduce(int* buff, const int* scratch, int rank, int nranks, size_t nelems,
                                       const void* channels4, void* gridBarrier, int nblocks, int nthreads,
                                       uint64_t budget, uint32_t* err, void* stream);
int mscclppAmdLaunchHostOffloadKernel(int rank, int nranks, const void* fifoHandle, void* semHandles, int handleIndex,
                                      uint64_t budget, uint32_t* err, void* stream);
int mscclppAmdLaunchPortChannelPut(void* chans, int nchans, const uint64_t* dstOffs, const uint64_t* srcOffs,
                                   uint64_t chunk, int mode, void* stream);

/* MemoryChannel device-surface self-test on one GPU (two in-process ranks): mode 0 LL16 packet
 * ping-pong, 1 LL8 ping-pong, 2 put + signal/wait round trip.  *failures = mismatching words.
 * Modes 3 / 4: rank 0 unpacks LL16 / LL8 packets of flag 7 that rank 1 never puts; the wait ends at
 * a 20 ms budget and devErr[0..3] (4 words) receives the error record (code, flag, packet byte,
 * flag seen). */
int mscclppAmdMemChannelSelfTest(int mode, int nElem, int nTries, int* failures, uint32_t* devErr);
/* put, get and putPackets + unpackPackets (LL16, LL8) of `bytes` (multiple of 16, meant to exceed
 * 4 GiB) on one GPU, nblocks x 256 lanes as one thread group; bad[0..3] = words that differ from the
 * source pattern after each of the four (memory_channel_device.hpp:101-215 take 64-bit offsets). */
int mscclppAmdMemChannelBigTest(uint64_t bytes, int nblocks, unsigned long long* bad, uint32_t* devErr);
/* The reference's MemoryChannel packet ping-pong latency (test/mp_unit/memory_channel_tests.cu:
 * 98-107), collective over a 2-rank communicator: a MemoryChannel into the peer's packet buffer built
 * with the host API, 1000 checked tries, then `iters` timed one-way hand-offs of nElem ints as LL8
 * (ll8 != 0) or LL16 packets.  out[0] = us per iteration (host clock between the barriers around the
 * launch), out[1] = 1 if every receive matched and no device error was recorded, out[2..5] (when
 * outLen allows) = the error record: code, flag, packet byte, flag seen. */
int mscclppAmdMemChannelPingPong(ncclComm_t comm, int nElem, int iters, int ll8, double* out, int outLen);
/* One rank's ping-pong kernel: `handle` = a host MemoryChannelDeviceHandle (dst_ = the peer's packet
 * buffer, packetBuffer_ = this rank's), rank 0 or 1, flags flagBase + 1 ... flagBase + nTries,
 * *ret = 1 on a mismatch. */
int mscclppAmdLaunchMemChannelPingPong(const void* handle, int* buff, int rank, int nElem, int nTries,
                                       uint32_t flagBase, int ll8, int* ret, void* stream);

/* ---- bootstrap (TcpBootstrap, src/core/bootstrap/bootstrap.cc:169-611) -------------------------
 * Host-only setup plane; uniqueId is the 128-byte ncclUniqueId from ncclGetUniqueId. */
int mscclppAmdBootstrapCreate(int rank, int nranks, const void* uniqueId, void** handle);
int mscclppAmdBootstrapAllGather(void* handle, const void* sendbuf, void* recvbuf, size_t bytes);
int mscclppAmdBootstrapBarrier(void* handle);
int mscclppAmdBootstrapDestroy(void* handle);

#ifdef __cplusplus
}
#endif

#endif /* MSCCLPP_AMD_H_ */
