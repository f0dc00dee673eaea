/*
 * NCCL-compatible C ABI exported by libmscclpp_amd.so (drop-in for libmscclpp_nccl.so on MI355X).
 *
 * Mirrors the reference's include/mscclpp/ext/nccl/nccl.h: the unique id (nccl.h:21-24), the
 * result codes (:27-37), ncclRedOp_t (:217-233) and ncclDataType_t (:236-253) keep their values
 * so that binaries built against nccl.h / rccl.h link and run unchanged.  Each entry point below
 * cites the reference function it replaces (src/ext/nccl/nccl.cc).
 *
 * Plain C types only: hipStream_t is carried as an opaque pointer.
 */
#ifndef MSCCLPP_AMD_NCCL_H_
#define MSCCLPP_AMD_NCCL_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NCCL_MAJOR 2
#define NCCL_MINOR 26
#define NCCL_PATCH 0
#define NCCL_VERSION_CODE 22600

typedef struct ncclComm* ncclComm_t;
#define NCCL_COMM_NULL NULL
typedef struct ncclWindow* ncclWindow_t; /* nccl.h:18 */

#define NCCL_UNIQUE_ID_BYTES 128
typedef struct {
  char internal[NCCL_UNIQUE_ID_BYTES];
} ncclUniqueId;

typedef enum {
  ncclSuccess = 0,
  ncclUnhandledCudaError = 1,
  ncclSystemError = 2,
  ncclInternalError = 3,
  ncclInvalidArgument = 4,
  ncclInvalidUsage = 5,
  ncclRemoteError = 6,
  ncclInProgress = 7,
  ncclNumResults = 8
} ncclResult_t;

typedef enum { ncclNumOps_dummy = 5 } ncclRedOp_dummy_t;
typedef enum {
  ncclSum = 0,
  ncclProd = 1,
  ncclMax = 2,
  ncclMin = 3,
  ncclAvg = 4,
  ncclNumOps = 5,
  ncclMaxRedOp = 0x7fffffff >> (32 - 8 * sizeof(ncclRedOp_dummy_t))
} ncclRedOp_t;

typedef enum {
  ncclInt8 = 0,
  ncclChar = 0,
  ncclUint8 = 1,
  ncclInt32 = 2,
  ncclInt = 2,
  ncclUint32 = 3,
  ncclInt64 = 4,
  ncclUint64 = 5,
  ncclFloat16 = 6,
  ncclHalf = 6,
  ncclFloat32 = 7,
  ncclFloat = 7,
  ncclFloat64 = 8,
  ncclDouble = 8,
  ncclBfloat16 = 9,
  ncclFloat8e4m3 = 10,
  ncclFloat8e5m2 = 11,
  ncclNumTypes = 12
} ncclDataType_t;

typedef struct ncclConfig_v21700 {
  size_t size;
  unsigned int magic;
  unsigned int version;
  int blocking;
  int cgaClusterSize;
  int minCTAs;
  int maxCTAs;
  const char* netName;
  int splitShare;
} ncclConfig_t;

#define NCCL_SPLIT_NOCOLOR -1

typedef enum { ncclScalarDevice = 0, ncclScalarHostImmediate = 1 } ncclScalarResidence_t;

typedef struct ncclSimInfo_v22200 {
  size_t size;
  unsigned int magic;
  unsigned int version;
  float estimatedTime;
} ncclSimInfo_t;

/* nccl.cc:187 */ ncclResult_t ncclGetVersion(int* version);
/* nccl.cc:196 */ ncclResult_t ncclGetUniqueId(ncclUniqueId* uniqueId);
/* nccl.cc:281 */ ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId commId, int rank);
/* nccl.cc:207 */ ncclResult_t ncclCommInitRankConfig(ncclComm_t* comm, int nranks, ncclUniqueId commId, int rank,
                                                      ncclConfig_t* config);
/* nccl.cc:351 */ ncclResult_t ncclCommInitAll(ncclComm_t* comm, int ndev, const int* devlist);
/* nccl.cc:362 */ ncclResult_t ncclCommFinalize(ncclComm_t comm);
/* nccl.cc:378 */ ncclResult_t ncclCommDestroy(ncclComm_t comm);
/* nccl.cc:400 */ ncclResult_t ncclCommAbort(ncclComm_t comm);
/* nccl.cc:442 */ const char* ncclGetErrorString(ncclResult_t result);
/* nccl.cc:465 */ const char* ncclGetLastError(ncclComm_t comm);
/* nccl.cc:470 */ ncclResult_t ncclCommGetAsyncError(ncclComm_t comm, ncclResult_t* asyncError);
/* nccl.cc:479 */ ncclResult_t ncclCommCount(const ncclComm_t comm, int* count);
/* nccl.cc:488 */ ncclResult_t ncclCommCuDevice(const ncclComm_t comm, int* device);
/* nccl.cc:497 */ ncclResult_t ncclCommUserRank(const ncclComm_t comm, int* rank);
/* nccl.cc:607 */ ncclResult_t ncclAllReduce(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype,
                                             ncclRedOp_t op, ncclComm_t comm, void* stream);
/* nccl.cc:662 */ ncclResult_t ncclReduceScatter(const void* sendbuff, void* recvbuff, size_t recvcount,
                                                 ncclDataType_t datatype, ncclRedOp_t op, ncclComm_t comm, void* stream);
/* nccl.cc:718 */ ncclResult_t ncclAllGather(const void* sendbuff, void* recvbuff, size_t sendcount,
                                             ncclDataType_t datatype, ncclComm_t comm, void* stream);
/* Native zero-copy pull from the root over xGMI (nccl.cc:544-605). */
/* nccl.cc:549 */ ncclResult_t ncclBroadcast(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype,
                                             int root, ncclComm_t comm, void* stream);
/* nccl.cc:544 */ ncclResult_t ncclBcast(void* buff, size_t count, ncclDataType_t datatype, int root, ncclComm_t comm,
                                         void* stream);
/* nccl.cc:405 -- a new communicator per color over the same bootstrap, ranks ordered by key */
/* nccl.cc:405 */ ncclResult_t ncclCommSplit(ncclComm_t comm, int color, int key, ncclComm_t* newcomm,
                                             ncclConfig_t* config);
/* Not carried by this path: forwarded to the vendor library named by MSCCLPP_AMD_NCCL_LIB_PATH
 * (the reference's MSCCLPP_NCCL_LIB_PATH fallback, nccl.cc:84-124, :331-346) when it is set,
 * otherwise they return ncclInvalidUsage (one rank: a local copy where the operation defines one). */
/* nccl.cc:533 */ ncclResult_t ncclReduce(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype,
                                          ncclRedOp_t op, int root, ncclComm_t comm, void* stream);
/* nccl.cc:774 */ ncclResult_t ncclSend(const void* sendbuff, size_t count, ncclDataType_t datatype, int peer,
                                        ncclComm_t comm, void* stream);
/* nccl.cc:784 */ ncclResult_t ncclRecv(void* recvbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                                        void* stream);
/* nccl.cc:794 */ ncclResult_t ncclAllToAll(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype,
                                            ncclComm_t comm, void* stream);
/* nccl.cc:808 */ ncclResult_t ncclAllToAllv(const void* sendbuff, const size_t sendcounts[], const size_t sdispls[],
                                             void* recvbuff, const size_t recvcounts[], const size_t rdispls[],
                                             ncclDataType_t datatype, ncclComm_t comm, void* stream);
/* nccl.cc:521 */ ncclResult_t ncclRedOpCreatePreMulSum(ncclRedOp_t* op, void* scalar, ncclDataType_t datatype,
                                                        ncclScalarResidence_t residence, ncclComm_t comm);
/* nccl.cc:527 */ ncclResult_t ncclRedOpDestroy(ncclRedOp_t op, ncclComm_t comm);
/* nccl.cc:437 */ ncclResult_t ncclCommInitRankScalable(ncclComm_t* newcomm, int nranks, int myrank, int nId,
                                                        ncclUniqueId* commIds, ncclConfig_t* config);
/* nccl.cc:840 */ ncclResult_t ncclGroupSimulateEnd(ncclSimInfo_t* simInfo);
/* nccl.cc:846 */ ncclResult_t ncclCommRegister(const ncclComm_t comm, void* buff, size_t size, void** handle);
/* nccl.cc:852 */ ncclResult_t ncclCommDeregister(const ncclComm_t comm, void* handle);
/* nccl.cc:511 / :516 (unavailable there): the path maps buffers lazily on first use, so a window is
 * the buffer's address handed back, as ncclCommRegister does; deregistering it is a no-op. */
/* nccl.cc:511 */ ncclResult_t ncclCommWindowRegister(ncclComm_t comm, void* buff, size_t size, ncclWindow_t* win,
                                                      int winFlags);
/* nccl.cc:516 */ ncclResult_t ncclCommWindowDeregister(ncclComm_t comm, ncclWindow_t win);
/* nccl.cc:823 */ ncclResult_t ncclGroupStart(void);
/* nccl.cc:832 */ ncclResult_t ncclGroupEnd(void);
/* nccl.cc:858 */ ncclResult_t ncclMemAlloc(void** ptr, size_t size);
/* nccl.cc:889 */ ncclResult_t ncclMemFree(void* ptr);

#ifdef __cplusplus
}
#endif

#endif /* MSCCLPP_AMD_NCCL_H_ */
