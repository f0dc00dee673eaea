// mscclpp_amd C++ algorithm plugin interface (host only).
//
// Mirrors the reference's plugin API for the collective path, so code written against it ports by
// changing the namespace:
//   mscclpp::Algorithm / AlgorithmBuilder / NativeAlgorithm / DslAlgorithm / AlgorithmCtxKey /
//   CollectiveRequest / AlgoSelectFunc / AlgorithmCollection   include/mscclpp/algorithm.hpp:14-350
//   mscclpp::collective::AlgorithmCollectionBuilder            include/mscclpp/ext/collectives/
//                                                              algorithm_collection_builder.hpp:23-66
//   mscclpp::DataType                                          include/mscclpp/gpu_data_types.hpp:170-183
// and the NCCL entry points of libmscclpp_amd.so dispatch through it exactly as nccl.cc does
// (nccl.cc:296-315 builds the collection at ncclCommInitRank, :586-596 selects and executes): a
// user registers builders and selectors on AlgorithmCollectionBuilder::getInstance() BEFORE
// ncclCommInitRank, and ncclAllReduce / ncclAllGather / ncclReduceScatter then run the algorithm
// the user's selector returns, or the built-in one the fallback selector picks.
//
// Differences from the reference, all in the MI355X direction: Communicator is a thin handle over
// ncclComm_t (one process per GPU; registerMemory maps a buffer of every rank over xGMI by IPC, the
// role of registerMemory + sendMemory/recvMemory in communicator.cc), streams are hipStream_t, and
// the Executor / ExecutionPlan classes wrap the C ABI of include/mscclpp_amd/executor.h.
#ifndef MSCCLPP_AMD_ALGORITHM_HPP_
#define MSCCLPP_AMD_ALGORITHM_HPP_

#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "mscclpp_amd/core.hpp"
#include "mscclpp_amd/executor.h"
#include "mscclpp_amd/nccl.h"

namespace mscclpp_amd {

// gpu_data_types.hpp:170-183 (same values)
enum class DataType {
  INT32,
  UINT32,
  FLOAT16,
  FLOAT32,
  BFLOAT16,
  FLOAT8_E4M3FN,
  FLOAT8_E4M3FNUZ,
  FLOAT8_E5M2,
  FLOAT8_E5M2FNUZ,
  UINT8,
  FLOAT8_E4M3B15,
  AUTO = 255,
};

// algorithm.hpp:19-45 (same values; CommResult casts to ncclResult_t, algorithm.hpp:31-41)
enum class CollectiveBufferMode { Any = 0, InPlace, OutOfPlace };
enum class AlgorithmType { Native = 0, DSL };
enum class CommResult {
  CommSuccess = 0,
  CommUnhandledCudaError = 1,
  CommSystemError = 2,
  CommInternalError = 3,
  CommInvalidArgument = 4,
  CommInvalidUsage = 5,
  CommRemoteError = 6,
  CommInProgress = 7,
  CommNumResults = 8
};
enum ReduceOp { SUM = 0, MIN = 3, NOP = 255 };

// ncclDataType_t -> DataType (datatype_conversion.hpp); AUTO for types the path does not carry.
DataType dataTypeFromNccl(ncclDataType_t t);

// The communicator handed to algorithms (the reference passes std::shared_ptr<mscclpp::Communicator>)
// is mscclpp_amd::Communicator of core.hpp.

// executor.hpp:15-18
enum class PacketType {
  LL8,   // 8-byte low-latency packet
  LL16,  // 16-byte low-latency packet
};

class ExecutionPlan {
 public:
  ExecutionPlan(const std::string& planPath, int rank);  // executor.hpp:30; throws on a bad plan
  ~ExecutionPlan();
  ExecutionPlan(const ExecutionPlan&) = delete;
  ExecutionPlan& operator=(const ExecutionPlan&) = delete;
  std::string name() const;
  std::string collective() const;
  size_t minMessageSize() const;
  size_t maxMessageSize() const;
  bool isInPlace() const;
  mscclppAmdExecutionPlan_t handle() const { return plan_; }

 private:
  mscclppAmdExecutionPlan_t plan_ = nullptr;
};

// executor.hpp:58-85.  execute() throws mscclpp_amd::Error on failure (the reference's behaviour);
// the scratch the plans use comes from the communicator (defaultScratchBuffer is accepted and unused).
class Executor {
 public:
  explicit Executor(std::shared_ptr<Communicator> comm, std::shared_ptr<char> defaultScratchBuffer = nullptr);
  ~Executor();
  Executor(const Executor&) = delete;
  Executor& operator=(const Executor&) = delete;
  void execute(int rank, void* sendbuff, void* recvBuff, size_t sendBuffSize, size_t recvBuffSize, DataType dataType,
               const ExecutionPlan& plan, hipStream_t stream, PacketType packetType = PacketType::LL16);
  void reset();

 private:
  std::shared_ptr<Communicator> comm_;  // kept alive for the executor's lifetime, as the reference does
  mscclppAmdExecutor_t ex_ = nullptr;
};

// algorithm.hpp:54-118
class Algorithm {
 public:
  struct Constraint {
    int worldSize;
    int nRanksPerNode;
  };
  virtual ~Algorithm() = default;
  virtual const std::string& name() const = 0;
  virtual const std::string& collective() const = 0;
  virtual const std::pair<size_t, size_t>& messageRange() const = 0;
  virtual const std::unordered_map<std::string, uint64_t>& tags() const = 0;
  virtual const CollectiveBufferMode& bufferMode() const = 0;
  virtual AlgorithmType type() const = 0;
  virtual Constraint constraint() const = 0;
  virtual void setMessageSizeRange(size_t minMessageSize, size_t maxMessageSize) = 0;
  virtual CommResult execute(std::shared_ptr<Communicator> comm, const void* input, void* output, size_t inputSize,
                             size_t outputSize, DataType dtype, ReduceOp op, hipStream_t stream,
                             std::shared_ptr<Executor> executor, int nBlocks = 0, int nThreadsPerBlock = 0,
                             bool symmetricMemory = false,
                             const std::unordered_map<std::string, uintptr_t>& extras = {},
                             DataType accumDtype = DataType::AUTO) = 0;
  virtual void reset() = 0;
};

class AlgorithmBuilder {
 public:
  virtual ~AlgorithmBuilder() = default;
  virtual std::shared_ptr<Algorithm> build() = 0;
};

// algorithm.hpp:136-165
struct AlgorithmCtxKey {
  void* baseSendBuff;
  void* baseRecvBuff;
  size_t baseSendSize;
  size_t baseRecvSize;
  int tag;
  bool operator==(const AlgorithmCtxKey& o) const {
    return baseSendBuff == o.baseSendBuff && baseRecvBuff == o.baseRecvBuff && baseSendSize == o.baseSendSize &&
           baseRecvSize == o.baseRecvSize && tag == o.tag;
  }
};

struct AlgorithmCtxKeyHash {
  size_t operator()(const AlgorithmCtxKey& k) const;
};

// algorithm.hpp:170-262: context cached per AlgorithmCtxKey; InitFunc runs once, on first execute.
class NativeAlgorithm : public Algorithm {
 public:
  using InitFunc = std::function<void(std::shared_ptr<Communicator>)>;
  using KernelFunc =
      std::function<CommResult(const std::shared_ptr<void>, const void*, void*, size_t, size_t, DataType, ReduceOp,
                               hipStream_t, int, int, const std::unordered_map<std::string, uintptr_t>&, DataType)>;
  using ContextInitFunc =
      std::function<std::shared_ptr<void>(std::shared_ptr<Communicator>, const void*, void*, size_t, size_t, DataType)>;
  using ContextKeyGenFunc = std::function<AlgorithmCtxKey(const void* input, void* output, size_t inputSize,
                                                          size_t outputSize, DataType dtype, bool symmetricMemory)>;

  NativeAlgorithm(std::string name, std::string collective, InitFunc initFunc, KernelFunc kernelFunc,
                  ContextInitFunc contextInitFunc, ContextKeyGenFunc contextKeyGenFunc, size_t minMessageSize = 0,
                  size_t maxMessageSize = UINT64_MAX, CollectiveBufferMode bufferMode = CollectiveBufferMode::Any,
                  std::unordered_map<std::string, uint64_t> tags = {}, Constraint constraint = {});

  CommResult execute(std::shared_ptr<Communicator> comm, const void* input, void* output, size_t inputSize,
                     size_t outputSize, DataType dtype, ReduceOp op, hipStream_t stream,
                     std::shared_ptr<Executor> executor, int nBlocks = 0, int nThreadsPerBlock = 0,
                     bool symmetricMemory = false, const std::unordered_map<std::string, uintptr_t>& extras = {},
                     DataType accumDtype = DataType::AUTO) override;
  const std::string& name() const override { return name_; }
  const std::string& collective() const override { return collective_; }
  const std::pair<size_t, size_t>& messageRange() const override { return range_; }
  void setMessageSizeRange(size_t minMessageSize, size_t maxMessageSize) override {
    range_ = {minMessageSize, maxMessageSize};
  }
  const std::unordered_map<std::string, uint64_t>& tags() const override { return tags_; }
  const CollectiveBufferMode& bufferMode() const override { return bufferMode_; }
  AlgorithmType type() const override { return AlgorithmType::Native; }
  Constraint constraint() const override { return constraint_; }
  void reset() override { contexts_.clear(); }
  size_t numContexts() const { return contexts_.size(); }

 private:
  std::string name_, collective_;
  InitFunc initFunc_;
  KernelFunc kernelFunc_;
  ContextInitFunc contextInitFunc_;
  ContextKeyGenFunc contextKeyGenFunc_;
  std::pair<size_t, size_t> range_;
  CollectiveBufferMode bufferMode_;
  std::unordered_map<std::string, uint64_t> tags_;
  Constraint constraint_;
  std::unordered_map<AlgorithmCtxKey, std::shared_ptr<void>, AlgorithmCtxKeyHash> contexts_;
  bool initialized_ = false;
};

// algorithm.hpp:269-300: an execution plan run by the Executor passed to execute().
class DslAlgorithm : public Algorithm, public AlgorithmBuilder, public std::enable_shared_from_this<DslAlgorithm> {
 public:
  DslAlgorithm(std::string id, std::shared_ptr<ExecutionPlan> plan, std::unordered_map<std::string, uint64_t> tags = {},
               Constraint constraint = {});
  const std::string& name() const override { return name_; }
  const std::string& collective() const override { return collective_; }
  const std::pair<size_t, size_t>& messageRange() const override { return range_; }
  void setMessageSizeRange(size_t minMessageSize, size_t maxMessageSize) override {
    range_ = {minMessageSize, maxMessageSize};
  }
  const std::unordered_map<std::string, uint64_t>& tags() const override { return tags_; }
  const CollectiveBufferMode& bufferMode() const override { return bufferMode_; }
  AlgorithmType type() const override { return AlgorithmType::DSL; }
  Constraint constraint() const override { return constraint_; }
  CommResult execute(std::shared_ptr<Communicator> comm, const void* input, void* output, size_t inputSize,
                     size_t outputSize, DataType dtype, ReduceOp op, hipStream_t stream,
                     std::shared_ptr<Executor> executor, int nBlocks = 0, int nThreadsPerBlock = 0,
                     bool symmetricMemory = false, const std::unordered_map<std::string, uintptr_t>& extras = {},
                     DataType accumDtype = DataType::AUTO) override;
  void reset() override {}
  std::shared_ptr<Algorithm> build() override { return shared_from_this(); }
  const std::string& id() const { return id_; }

 private:
  std::shared_ptr<ExecutionPlan> plan_;
  std::string id_, name_, collective_;
  std::pair<size_t, size_t> range_;
  CollectiveBufferMode bufferMode_;
  std::unordered_map<std::string, uint64_t> tags_;
  Constraint constraint_;
};

// algorithm.hpp:302-319
struct CollectiveRequest {
  int worldSize;
  int nRanksPerNode;
  int rank;
  const void* inputBuffer;
  void* outputBuffer;
  size_t messageSize;
  hipStream_t stream;
  const std::string& collective;
  const DataType dtype;
  const std::unordered_map<std::string, std::vector<uint64_t>>& hints;
  CollectiveBufferMode bufferMode() const;  // algorithm.cc:13-24
};

using AlgoMapByCollective =
    std::unordered_map<std::string, std::unordered_map<std::string, std::shared_ptr<Algorithm>>>;
using AlgoSelectFunc = std::function<std::shared_ptr<Algorithm>(const AlgoMapByCollective&, const CollectiveRequest&)>;

// algorithm.hpp:326-368
class AlgorithmCollection {
 public:
  // The primary selector first; the fallback when it returns nullptr.  No selector at all is an
  // invalid usage (algorithm.cc:98-110): throws std::logic_error (ncclInvalidUsage at the ABI).
  std::shared_ptr<Algorithm> selectAlgorithm(const CollectiveRequest& request);
  void registerAlgorithm(const std::string collective, const std::string algoName, std::shared_ptr<Algorithm> algorithm);
  std::unordered_map<std::string, std::shared_ptr<Algorithm>> getAlgorithmsByCollective(
      const std::string& collective) const;
  std::vector<std::shared_ptr<Algorithm>> getAllAlgorithms() const;
  void extend(const AlgorithmCollection& other);
  void setSelectors(AlgoSelectFunc algoSelector, AlgoSelectFunc fallbackAlgoSelector);
  bool hasAlgorithmSelector() const { return (bool)algoSelector_; }  // a user's primary selector is set

 private:
  AlgoMapByCollective algoMapByCollective_;
  AlgoSelectFunc algoSelector_ = nullptr;
  AlgoSelectFunc fallbackAlgoSelector_ = nullptr;
};

// The built-in selector for one MI355X node (algorithm_selector.cc:91-161, AMD branch):
// allreduce <= 16 KiB default_allreduce_allpair_packet, <= 1 MiB default_allreduce_packet, larger
// default_allreduce_fullmesh (MSCCLPP_AMD_ALGO=<name> forces one); allgather
// default_allgather_fullmesh2; reducescatter default_reducescatter_fullmesh.
std::shared_ptr<Algorithm> defaultAlgoSelector(const AlgoMapByCollective& algoMap, const CollectiveRequest& request);

namespace collective {

// algorithm_collection_builder.hpp:23-66 / algorithm_collection_builder.cc
class AlgorithmCollectionBuilder {
 public:
  static std::shared_ptr<AlgorithmCollectionBuilder> getInstance();
  static void reset();
  void addAlgorithmBuilder(std::shared_ptr<AlgorithmBuilder> builder);
  void setAlgorithmSelector(AlgoSelectFunc selector);
  void setFallbackAlgorithmSelector(AlgoSelectFunc selector);
  // The user-registered algorithms, with the builder's selectors.
  AlgorithmCollection build();
  // The built-in native algorithms of this library for communicator `comm` (the reference passes
  // the communicator's scratch and flag buffers; here the communicator owns them), with the
  // builder's selectors.
  AlgorithmCollection buildDefaultAlgorithms(ncclComm_t comm);

 private:
  AlgorithmCollectionBuilder() = default;
  std::vector<std::shared_ptr<AlgorithmBuilder>> algoBuilders_;
  AlgoSelectFunc algoSelector_ = nullptr;
  AlgoSelectFunc fallbackAlgoSelector_ = nullptr;
};

}  // namespace collective
}  // namespace mscclpp_amd

#endif  // MSCCLPP_AMD_ALGORITHM_HPP_
