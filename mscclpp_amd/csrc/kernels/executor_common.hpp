// Execution-plan structures shared by the host executor and the device interpreter.
//
// Reference: src/core/include/execution_common.hpp:12-157 (OperationType, BufferType, Operation,
// DeviceExecutionPlan).  The operation codes keep the reference's numbering so plans, traces and
// tools agree; the layout is this build's own: 64-bit offsets and sizes (buffers on a 288 GB GPU
// can pass 4 GiB), per-channel semaphore pointers instead of DeviceHandle objects, and one
// threadblock plan = header + operations, copied into LDS by its workgroup at kernel start.
#pragma once

#include <stdint.h>

namespace mscclpp_amd {
namespace exec {

constexpr int kMaxBuffersPerOp = 10;  // MAX_LOCAL_BUFFER_PER_OPERATION + MAX_CHANNEL_PER_OPERATION
constexpr int kMaxChannelsPerOp = 8;  // MAX_CHANNEL_PER_OPERATION
constexpr int kMaxChannels = 16;      // per threadblock (MAX_CHANNEL)
constexpr int kMaxOps = 128;          // per threadblock (reference MAX_OPERATION = 64)
constexpr int kMaxSyncers = 16;       // MAX_DEVICE_SYNCERS
constexpr int kMaxSemaphores = 16;    // MAX_DEVICE_SEMAPHORES
constexpr int kMaxTags = 64;          // memory channels between one pair of ranks
constexpr int kMaxRanks = 8;

// execution_common.hpp:40-71, same order
enum OpType : uint8_t {
  NOP,
  BARRIER,
  PUT,
  PUT_PACKETS,
  READ_PUT_PACKETS,
  PUT_WITH_SIGNAL,
  PUT_WITH_SIGNAL_AND_FLUSH,
  GET,
  COPY,
  COPY_PACKETS,
  UNPACK_PACKETS,
  SIGNAL,
  WAIT,
  FLUSH,
  REDUCE,
  REDUCE_PACKETS,
  REDUCE_COPY_PACKETS,
  REDUCE_SEND,
  REDUCE_SEND_PACKETS,
  REDUCE_COPY_SEND_PACKETS,
  READ_REDUCE,
  READ_REDUCE_SEND,
  MULTI_LOAD_REDUCE_STORE,
  RELAXED_SIGNAL,
  RELAXED_WAIT,
  PIPELINE,
  SEM_RELEASE,
  SEM_ACQUIRE,
  MULTI_STORE,
  MULTI_STORE_PKT,
};

// execution_common.hpp:22-27
enum BufType : uint8_t { kInput = 0, kOutput = 1, kScratch = 2, kNoBuffer = 0xFF };

struct Op {
  uint8_t type;
  uint8_t nInputs;
  uint8_t nOutputs;
  uint8_t nChannels;
  uint8_t reduceOp;  // 0 sum, 1 min
  uint8_t nSems;
  uint8_t pad[2];
  // per buffer slot: a local BufType, or (for slots addressed through a channel) the index into
  // the threadblock's remote buffer table
  uint8_t inRef[kMaxBuffersPerOp];
  uint8_t outRef[kMaxBuffersPerOp];
  uint8_t chan[kMaxChannelsPerOp];
  uint8_t semIds[kMaxSemaphores];
  uint32_t syncer;         // BARRIER: syncer index
  uint32_t nThreadBlocks;  // BARRIER: workgroups that meet
  uint32_t nIterations;    // PIPELINE
  uint32_t nOperations;    // PIPELINE: inner operations that follow
  uint64_t unitSize;       // PIPELINE
  uint64_t inOff[kMaxBuffersPerOp];
  uint64_t outOff[kMaxBuffersPerOp];
  uint64_t inSize[kMaxBuffersPerOp];
  uint64_t outSize[kMaxBuffersPerOp];
};

// A memory channel as the device sees it (MemoryDevice2DeviceSemaphore, semaphore_device.hpp:61-135)
struct Chan {
  uint64_t* remoteToken;  // my slot in the peer's inbound tokens
  uint64_t* inbound;      // the peer's slot in my inbound tokens
  uint64_t* expected;     // my wait counter for that slot
};

struct TbHeader {
  uint32_t nOps;
  uint32_t nChannels;
  uint32_t nRemote;
  uint32_t pad;
  Chan ch[kMaxChannels];
  void* remotePtr[kMaxChannels];       // remote buffers (peer pointers mapped here)
  uint8_t remoteType[kMaxChannels];    // their BufType
};

struct TbPlan {
  TbHeader h;
  Op ops[kMaxOps];
};

// Cross-workgroup barrier (DeviceSyncer, concurrency_device.hpp) and counting semaphore
// (DeviceSemaphore): both live in device memory owned by the executor.
struct Syncer {
  uint64_t count;  // monotonic: every arrival adds 1
  uint64_t pad[7];
};

struct Sem {
  int64_t value;
  int64_t pad[7];
};

}  // namespace exec
}  // namespace mscclpp_amd
