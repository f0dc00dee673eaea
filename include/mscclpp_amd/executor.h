/* mscclpp_amd execution plans and executor: C ABI.
 *
 * Replaces the reference's C++ classes mscclpp::ExecutionPlan and mscclpp::Executor
 * (include/mscclpp/executor.hpp:21-99, src/core/executor/execution_plan.cc,
 * src/core/executor/executor.cc).  A plan is the reference's JSON plan format (the output of the
 * mscclpp DSL, e.g. test/execution-files/allreduce_packet.json); the executor runs it on a
 * communicator created with ncclCommInitRank.  Every rank of the communicator must call
 * mscclppAmdExecutorExecute for the same plan, in the same order (setup is collective).
 *
 * Supported operations: nop, barrier, signal/wait, rlxsignal/rlxwait, put/pws/pwsf, get, copy,
 * re/res/rre/rres, ppkt/rppkt/respkt/repkt/recspkt/recpkt/upkt/cpkt, sem_acquire/sem_release and
 * pipeline over memory channels.  Port channels and NVLS ("switch") channels are rejected when the
 * plan is loaded: plans for one MI355X node use memory channels over xGMI.
 */
#ifndef MSCCLPP_AMD_EXECUTOR_H_
#define MSCCLPP_AMD_EXECUTOR_H_

#include <stddef.h>
#include <stdint.h>

#include "mscclpp_amd/nccl.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mscclppAmdExecutionPlan* mscclppAmdExecutionPlan_t;
typedef struct mscclppAmdExecutor* mscclppAmdExecutor_t;

/* mscclpp::DataType values (include/mscclpp/gpu_data_types.hpp:169-183) */
enum {
  MSCCLPP_AMD_DT_INT32 = 0,
  MSCCLPP_AMD_DT_UINT32 = 1,
  MSCCLPP_AMD_DT_FLOAT16 = 2,
  MSCCLPP_AMD_DT_FLOAT32 = 3,
  MSCCLPP_AMD_DT_BFLOAT16 = 4,
  MSCCLPP_AMD_DT_FLOAT8_E4M3FN = 5,   /* OCP: gfx950's hardware format */
  MSCCLPP_AMD_DT_FLOAT8_E4M3FNUZ = 6, /* not native on gfx950: rejected, as the reference does */
  MSCCLPP_AMD_DT_FLOAT8_E5M2 = 7,     /* OCP */
  MSCCLPP_AMD_DT_FLOAT8_E5M2FNUZ = 8, /* not native on gfx950: rejected */
  MSCCLPP_AMD_DT_UINT8 = 9,
  MSCCLPP_AMD_DT_FLOAT8_E4M3B15 = 10, /* software fp8, bias 15 (execution_kernel.hpp:997-1007) */
};
/* mscclpp::PacketType (executor.hpp:15-18) */
enum { MSCCLPP_AMD_PACKET_LL8 = 0, MSCCLPP_AMD_PACKET_LL16 = 1 };

/* ExecutionPlan(planPath, rank) (executor.hpp:30, execution_plan.cc:124-135).  Returns
 * ncclInvalidArgument for an unreadable or malformed plan. */
int mscclppAmdExecutionPlanCreate(const char* planPath, int rank, mscclppAmdExecutionPlan_t* plan);
int mscclppAmdExecutionPlanDestroy(mscclppAmdExecutionPlan_t plan);
/* name() / collective() / minMessageSize() / maxMessageSize() / isInPlace() (executor.hpp:36-49) */
const char* mscclppAmdExecutionPlanName(mscclppAmdExecutionPlan_t plan);
const char* mscclppAmdExecutionPlanCollective(mscclppAmdExecutionPlan_t plan);
size_t mscclppAmdExecutionPlanMinMessageSize(mscclppAmdExecutionPlan_t plan);
size_t mscclppAmdExecutionPlanMaxMessageSize(mscclppAmdExecutionPlan_t plan);
int mscclppAmdExecutionPlanIsInPlace(mscclppAmdExecutionPlan_t plan);
/* Host-only lowering (no device work): the plan resolved for this rank at the given message sizes,
 * written as JSON text into buf (truncated to len; the full length is returned in *needed).  Lists
 * per threadblock the memory channels (peer, tag), remote buffers (peer, type) and each operation's
 * type, buffer references, byte offsets and sizes (setupOperation, execution_plan.cc:480-605). */
int mscclppAmdExecutionPlanDescribe(mscclppAmdExecutionPlan_t plan, size_t inputBytes, size_t outputBytes, char* buf,
                                    size_t len, size_t* needed);

/* Executor(comm) (executor.hpp:63-66).  Collective over the communicator. */
int mscclppAmdExecutorCreate(ncclComm_t comm, mscclppAmdExecutor_t* executor);
/* Executor::execute (executor.hpp:85-86): sendBytes / recvBytes are the message sizes, dtype an
 * MSCCLPP_AMD_DT_* value, stream a hipStream_t, packetType MSCCLPP_AMD_PACKET_*.  Returns 0, or
 * ncclInvalidArgument / ncclInvalidUsage for sizes or dtypes the plan cannot run. */
int mscclppAmdExecutorExecute(mscclppAmdExecutor_t executor, int rank, void* sendbuff, void* recvbuff, size_t sendBytes,
                              size_t recvBytes, int dtype, mscclppAmdExecutionPlan_t plan, void* stream,
                              int packetType);
/* Executor::reset (executor.hpp:92): drop cached contexts (collective). */
int mscclppAmdExecutorReset(mscclppAmdExecutor_t executor);
int mscclppAmdExecutorDestroy(mscclppAmdExecutor_t executor);
/* Device error word of the executor's kernels: code + three diagnostic words (0 = ok). */
int mscclppAmdExecutorGetDeviceError(mscclppAmdExecutor_t executor, uint32_t* words4, int clear);

#ifdef __cplusplus
}
#endif

#endif /* MSCCLPP_AMD_EXECUTOR_H_ */
