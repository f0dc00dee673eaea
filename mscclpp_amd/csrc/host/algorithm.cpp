// The C++ algorithm plugin layer (include/mscclpp_amd/algorithm.hpp) and the built-in algorithms
// the NCCL entry points dispatch to through it.
//
//   NativeAlgorithm::execute      src/core/algorithm.cc:42-68 (init once, context cache per key)
//   DslAlgorithm                  src/core/algorithm.cc:140-230 (plan run by the passed Executor)
//   AlgorithmCollection           src/core/algorithm.cc:92-136
//   CollectiveRequest::bufferMode src/core/algorithm.cc:13-24
//   AlgorithmCollectionBuilder    src/ext/collectives/algorithm_collection_builder.cc:20-70
//   defaultAlgoSelector           src/ext/nccl/algorithm_selector.cc:91-161 (AMD single-node branch)
#include "mscclpp_amd/algorithm.hpp"

#include <stdexcept>

#include "comm_internal.hpp"

namespace mscclpp_amd {

DataType dataTypeFromNccl(ncclDataType_t t) {
  switch (t) {
    case ncclInt32: return DataType::INT32;
    case ncclUint32: return DataType::UINT32;
    case ncclFloat16: return DataType::FLOAT16;
    case ncclFloat32: return DataType::FLOAT32;
    case ncclBfloat16: return DataType::BFLOAT16;
    case ncclFloat8e4m3: return DataType::FLOAT8_E4M3FN;  // OCP on gfx950
    case ncclFloat8e5m2: return DataType::FLOAT8_E5M2;
    case ncclUint8: return DataType::UINT8;
    default: return DataType::AUTO;
  }
}

// DataType (+ accumulation DataType) -> the kernels' reduce-type code, or -1.
static int reduceTypeOf(DataType dt, DataType accum) {
  if (accum == DataType::AUTO) accum = dt;
  switch (dt) {
    case DataType::FLOAT16: return accum == dt ? MSCCLPP_AMD_F16 : -1;
    case DataType::BFLOAT16: return accum == dt ? MSCCLPP_AMD_BF16 : -1;
    case DataType::FLOAT32: return accum == dt ? MSCCLPP_AMD_F32 : -1;
    case DataType::INT32: return accum == dt ? MSCCLPP_AMD_I32 : -1;
    case DataType::UINT32: return accum == dt ? MSCCLPP_AMD_U32 : -1;
    case DataType::FLOAT8_E4M3FN:
      return accum == dt                  ? MSCCLPP_AMD_E4M3
             : accum == DataType::FLOAT16 ? MSCCLPP_AMD_E4M3_ACC_F16
             : accum == DataType::FLOAT32 ? MSCCLPP_AMD_E4M3_ACC_F32
                                          : -1;
    case DataType::FLOAT8_E5M2:
      return accum == dt                  ? MSCCLPP_AMD_E5M2
             : accum == DataType::FLOAT16 ? MSCCLPP_AMD_E5M2_ACC_F16
             : accum == DataType::FLOAT32 ? MSCCLPP_AMD_E5M2_ACC_F32
                                          : -1;
    case DataType::UINT8: return accum == dt ? MSCCLPP_AMD_U8 : -1;
    case DataType::FLOAT8_E4M3B15:  // software on every platform (gpu_data_types.hpp:78-155)
      return accum == dt                  ? MSCCLPP_AMD_E4M3B15
             : accum == DataType::FLOAT16 ? MSCCLPP_AMD_E4M3B15_ACC_F16
             : accum == DataType::FLOAT32 ? MSCCLPP_AMD_E4M3B15_ACC_F32
                                          : -1;
    default: return -1;  // FNUZ: the reference's gfx950 build has no FNUZ kernels either (common.hpp:110-126)
  }
}

static CommResult asResult(int code) {
  return (code >= 0 && code < (int)CommResult::CommNumResults) ? (CommResult)code : CommResult::CommInternalError;
}

// ---- ExecutionPlan / Executor (C ABI wrappers) ------------------------------------------------
ExecutionPlan::ExecutionPlan(const std::string& planPath, int rank) {
  if (mscclppAmdExecutionPlanCreate(planPath.c_str(), rank, &plan_) != 0)
    throw std::invalid_argument("ExecutionPlan: cannot load " + planPath + ": " + ncclGetLastError(nullptr));
}
ExecutionPlan::~ExecutionPlan() {
  if (plan_) (void)mscclppAmdExecutionPlanDestroy(plan_);
}
std::string ExecutionPlan::name() const { return mscclppAmdExecutionPlanName(plan_); }
std::string ExecutionPlan::collective() const { return mscclppAmdExecutionPlanCollective(plan_); }
size_t ExecutionPlan::minMessageSize() const { return mscclppAmdExecutionPlanMinMessageSize(plan_); }
size_t ExecutionPlan::maxMessageSize() const { return mscclppAmdExecutionPlanMaxMessageSize(plan_); }
bool ExecutionPlan::isInPlace() const { return mscclppAmdExecutionPlanIsInPlace(plan_) != 0; }

Executor::Executor(std::shared_ptr<Communicator> comm, std::shared_ptr<char>) : comm_(comm) {
  if (!comm) throw Error("Executor: null communicator", ErrorCode::InvalidUsage);
  if (mscclppAmdExecutorCreate(comm->ncclComm(), &ex_) != 0)
    throw Error(std::string("Executor: ") + ncclGetLastError(nullptr), ErrorCode::InternalError);
}
Executor::~Executor() {
  if (ex_) (void)mscclppAmdExecutorDestroy(ex_);
}
void Executor::execute(int rank, void* sendbuff, void* recvbuff, size_t sendBuffSize, size_t recvBuffSize,
                       DataType dataType, const ExecutionPlan& plan, hipStream_t stream, PacketType packetType) {
  const int r = mscclppAmdExecutorExecute(ex_, rank, sendbuff, recvbuff, sendBuffSize, recvBuffSize, (int)dataType,
                                          plan.handle(), (void*)stream,
                                          packetType == PacketType::LL16 ? MSCCLPP_AMD_PACKET_LL16 : MSCCLPP_AMD_PACKET_LL8);
  if (r == ncclSuccess) return;
  const ErrorCode code = r == ncclInvalidArgument || r == ncclInvalidUsage ? ErrorCode::InvalidUsage
                         : r == ncclUnhandledCudaError || r == ncclSystemError ? ErrorCode::SystemError
                                                                               : ErrorCode::ExecutorError;
  throw Error(std::string("Executor::execute: ") + ncclGetLastError(nullptr), code);
}
void Executor::reset() { (void)mscclppAmdExecutorReset(ex_); }

// ---- NativeAlgorithm --------------------------------------------------------------------------
size_t AlgorithmCtxKeyHash::operator()(const AlgorithmCtxKey& k) const {
  size_t seed = 42;
  auto mix = [&](size_t v) { seed ^= v + 0x9e3779b97f4a7c15ull + (seed << 6) + (seed >> 2); };
  mix(std::hash<const void*>()(k.baseSendBuff));
  mix(std::hash<const void*>()(k.baseRecvBuff));
  mix(std::hash<size_t>()(k.baseSendSize));
  mix(std::hash<size_t>()(k.baseRecvSize));
  mix(std::hash<int>()(k.tag));
  return seed;
}

NativeAlgorithm::NativeAlgorithm(std::string name, std::string collective, InitFunc initFunc, KernelFunc kernelFunc,
                                 ContextInitFunc contextInitFunc, ContextKeyGenFunc contextKeyGenFunc,
                                 size_t minMessageSize, size_t maxMessageSize, CollectiveBufferMode bufferMode,
                                 std::unordered_map<std::string, uint64_t> tags, Constraint constraint)
    : name_(std::move(name)),
      collective_(std::move(collective)),
      initFunc_(std::move(initFunc)),
      kernelFunc_(std::move(kernelFunc)),
      contextInitFunc_(std::move(contextInitFunc)),
      contextKeyGenFunc_(std::move(contextKeyGenFunc)),
      range_(minMessageSize, maxMessageSize),
      bufferMode_(bufferMode),
      tags_(std::move(tags)),
      constraint_(constraint) {}

CommResult NativeAlgorithm::execute(std::shared_ptr<Communicator> comm, const void* input, void* output,
                                    size_t inputSize, size_t outputSize, DataType dtype, ReduceOp op,
                                    hipStream_t stream, std::shared_ptr<Executor>, int nBlocks, int nThreadsPerBlock,
                                    bool symmetricMemory, const std::unordered_map<std::string, uintptr_t>& extras,
                                    DataType accumDtype) {
  if (accumDtype == DataType::AUTO) accumDtype = dtype;
  if (!initialized_) {
    if (initFunc_) initFunc_(comm);
    initialized_ = true;
  }
  const AlgorithmCtxKey key = contextKeyGenFunc_(input, output, inputSize, outputSize, dtype, symmetricMemory);
  auto it = contexts_.find(key);
  if (it == contexts_.end())  // a miss is collective setup (every rank misses on the same call)
    it = contexts_.emplace(key, contextInitFunc_(comm, input, output, inputSize, outputSize, dtype)).first;
  return kernelFunc_(it->second, input, output, inputSize, outputSize, dtype, op, stream, nBlocks, nThreadsPerBlock,
                     extras, accumDtype);
}

// ---- DslAlgorithm -----------------------------------------------------------------------------
DslAlgorithm::DslAlgorithm(std::string id, std::shared_ptr<ExecutionPlan> plan,
                           std::unordered_map<std::string, uint64_t> tags, Constraint constraint)
    : plan_(std::move(plan)), id_(std::move(id)), tags_(std::move(tags)), constraint_(constraint) {
  if (!plan_) throw std::invalid_argument("DslAlgorithm: null plan");
  name_ = plan_->name();
  collective_ = plan_->collective();
  range_ = {plan_->minMessageSize(), plan_->maxMessageSize()};
  bufferMode_ = plan_->isInPlace() ? CollectiveBufferMode::InPlace : CollectiveBufferMode::OutOfPlace;
}

CommResult DslAlgorithm::execute(std::shared_ptr<Communicator> comm, const void* input, void* output,
                                 size_t inputSize, size_t outputSize, DataType dtype, ReduceOp, hipStream_t stream,
                                 std::shared_ptr<Executor> executor, int, int, bool,
                                 const std::unordered_map<std::string, uintptr_t>&, DataType) {
  if (!executor) throw std::logic_error("Executor is null in DslAlgorithm::execute");  // algorithm.cc:178-180
  if (dtype == DataType::AUTO) return CommResult::CommInvalidArgument;  // the executor checks the rest
  try {
    executor->execute(comm->rank(), const_cast<void*>(input), output, inputSize, outputSize, dtype, *plan_, stream);
  } catch (const Error& e) {
    return e.getErrorCode() == ErrorCode::InvalidUsage ? CommResult::CommInvalidArgument : CommResult::CommInternalError;
  }
  return CommResult::CommSuccess;
}

// ---- CollectiveRequest / AlgorithmCollection ---------------------------------------------------
CollectiveBufferMode CollectiveRequest::bufferMode() const {
  if (inputBuffer == outputBuffer) return CollectiveBufferMode::InPlace;
  if (collective == "allgather") {
    const char* expected = static_cast<const char*>(outputBuffer) + (size_t)rank * messageSize;
    return static_cast<const void*>(expected) == inputBuffer ? CollectiveBufferMode::InPlace
                                                             : CollectiveBufferMode::OutOfPlace;
  }
  return CollectiveBufferMode::OutOfPlace;
}

std::shared_ptr<Algorithm> AlgorithmCollection::selectAlgorithm(const CollectiveRequest& request) {
  if (!algoSelector_ && !fallbackAlgoSelector_)
    throw std::logic_error("No algorithm selector is set in AlgorithmCollection.");
  std::shared_ptr<Algorithm> algo;
  if (algoSelector_) algo = algoSelector_(algoMapByCollective_, request);
  if (!algo && fallbackAlgoSelector_) algo = fallbackAlgoSelector_(algoMapByCollective_, request);
  return algo;
}

void AlgorithmCollection::registerAlgorithm(const std::string collective, const std::string algoName,
                                            std::shared_ptr<Algorithm> algorithm) {
  algoMapByCollective_[collective][algoName] = std::move(algorithm);
}

std::unordered_map<std::string, std::shared_ptr<Algorithm>> AlgorithmCollection::getAlgorithmsByCollective(
    const std::string& collective) const {
  auto it = algoMapByCollective_.find(collective);
  if (it == algoMapByCollective_.end()) return {};
  return it->second;
}

std::vector<std::shared_ptr<Algorithm>> AlgorithmCollection::getAllAlgorithms() const {
  std::vector<std::shared_ptr<Algorithm>> all;
  for (const auto& c : algoMapByCollective_)
    for (const auto& a : c.second) all.push_back(a.second);
  return all;
}

void AlgorithmCollection::extend(const AlgorithmCollection& other) {
  for (const auto& c : other.algoMapByCollective_)
    for (const auto& a : c.second) registerAlgorithm(c.first, a.first, a.second);
}

void AlgorithmCollection::setSelectors(AlgoSelectFunc algoSelector, AlgoSelectFunc fallbackAlgoSelector) {
  algoSelector_ = std::move(algoSelector);
  fallbackAlgoSelector_ = std::move(fallbackAlgoSelector);
}

// ---- built-in algorithms ----------------------------------------------------------------------
namespace {

struct BuiltinCtx {
  ncclComm* comm;
};

// One built-in native algorithm: `code` is the launcher's algorithm (MSCCLPP_AMD_ALGO_*), `coll`
// 0 = AllReduce, 1 = ReduceScatter, 2 = AllGather (the bulk kernel's modes).  Contexts: the
// communicator itself caches scratch and per-buffer IPC mappings, so the per-key context is a
// handle to it and the key is the buffer pair (algorithm.cc:52-60).
std::shared_ptr<Algorithm> builtin(ncclComm* comm, const std::string& name, const std::string& collective, int code,
                                   int coll, size_t minBytes, size_t maxBytes) {
  auto kernel = [code, coll, name, collective](const std::shared_ptr<void> ctx, const void* in, void* out,
                                               size_t inSize, size_t outSize, DataType dtype, ReduceOp op,
                                               hipStream_t stream, int nBlocks, int nThreads,
                                               const std::unordered_map<std::string, uintptr_t>&,
                                               DataType accum) -> CommResult {
    ncclComm* c = std::static_pointer_cast<BuiltinCtx>(ctx)->comm;
    if (nBlocks == kTunedShapeResolved) {  // the caller looked the tuned shape up already: defaults
      nBlocks = 0;
    } else if (nBlocks <= 0 && nThreads <= 0) {  // the tuned launch shape of this algorithm, if any
      std::string tuned;
      int nb = 0, nt = 0;
      const size_t msg = inSize;  // the request's messageSize for all three (nccl.cc:586, :697, :748)
      if (tunedConfig(collective, c->nranks, msg, tuned, nb, nt) && tuned == name) {
        nBlocks = nb;
        nThreads = nt;
      }
    }
    if (coll == 2) {  // AllGather moves bytes: the element type only sets the unit
      if (inSize == 0 || outSize != inSize * (size_t)c->nranks) return CommResult::CommInvalidArgument;
      return asResult(c->bulkCollective(2, in, out, inSize, MSCCLPP_AMD_F32, MSCCLPP_AMD_SUM, code, nBlocks,
                                        nThreads, stream));
    }
    const int dt = reduceTypeOf(dtype, accum);
    const int o = op == SUM ? MSCCLPP_AMD_SUM : op == MIN ? MSCCLPP_AMD_MIN : -1;
    if (dt < 0 || o < 0) return CommResult::CommInvalidArgument;
    if (coll == 1) {
      if (outSize == 0 || inSize != outSize * (size_t)c->nranks) return CommResult::CommInvalidArgument;
      return asResult(c->bulkCollective(1, in, out, outSize, dt, o, code, nBlocks, nThreads, stream));
    }
    if (inSize == 0 || inSize != outSize) return CommResult::CommInvalidArgument;
    return asResult(c->allReduce(in, out, inSize, dt, o, code, nBlocks, nThreads, stream));
  };
  auto ctxInit = [comm](std::shared_ptr<Communicator>, const void*, void*, size_t, size_t, DataType) {
    return std::static_pointer_cast<void>(std::make_shared<BuiltinCtx>(BuiltinCtx{comm}));
  };
  auto key = [](const void* in, void* out, size_t inSize, size_t outSize, DataType, bool) {
    return AlgorithmCtxKey{const_cast<void*>(in), out, inSize, outSize, 0};
  };
  return std::make_shared<NativeAlgorithm>(name, collective, nullptr, kernel, ctxInit, key, minBytes, maxBytes,
                                           CollectiveBufferMode::Any,
                                           std::unordered_map<std::string, uint64_t>{{"default", 1}},
                                           Algorithm::Constraint{comm->nranks, comm->nranks});
}

// MSCCLPP_AMD_ALGO, read once (the reference reads its environment once, env.cpp).
const char* envAlgoName() {
  static const char* const name = []() -> const char* {
    const char* e = std::getenv("MSCCLPP_AMD_ALGO");
    if (!e || !*e) return nullptr;
    const std::string s(e);
    if (s == "packet") return "default_allreduce_packet";
    if (s == "allpair" || s == "allpair_packet") return "default_allreduce_allpair_packet";
    if (s == "fullmesh") return "default_allreduce_fullmesh";
    if (s == "rsag") return "default_allreduce_rsag";
    if (s == "rsag_zc" || s == "rsag_zero_copy") return "default_allreduce_rsag_zero_copy";
    if (s == "rsag_pipeline") return "default_allreduce_rsag_pipeline";
    return nullptr;
  }();
  return name;
}

std::shared_ptr<Algorithm> lookup(const AlgoMapByCollective& m, const std::string& coll, const char* name) {
  auto c = m.find(coll);
  if (c == m.end()) return nullptr;
  auto a = c->second.find(name);
  return a == c->second.end() ? nullptr : a->second;
}

}  // namespace

std::shared_ptr<Algorithm> defaultAlgoSelector(const AlgoMapByCollective& algoMap, const CollectiveRequest& request) {
  if (request.nRanksPerNode != request.worldSize) return nullptr;  // multi-node: not this path (:163-175)
  if (request.collective == "allreduce")
    if (const char* forced = envAlgoName()) return lookup(algoMap, "allreduce", forced);
  // the tuned-config store (tuning.cpp): user profiles for this SKU / rank count, then the built-in
  // table restating the AMD thresholds of algorithm_selector.cc:107-131
  std::string name;
  int nb = 0, nt = 0;
  if (tunedConfig(request.collective, request.worldSize, request.messageSize, name, nb, nt))
    if (auto a = lookup(algoMap, request.collective, name.c_str())) return a;
  if (request.collective == "allreduce") {
    const char* def = request.messageSize <= ((size_t)1 << 14)   ? "default_allreduce_allpair_packet"
                      : request.messageSize <= ((size_t)1 << 20) ? "default_allreduce_packet"
                                                                 : "default_allreduce_fullmesh";
    return lookup(algoMap, "allreduce", def);
  }
  if (request.collective == "allgather") return lookup(algoMap, "allgather", "default_allgather_fullmesh2");
  if (request.collective == "reducescatter")
    return lookup(algoMap, "reducescatter", "default_reducescatter_fullmesh");
  return nullptr;
}

namespace collective {

static std::shared_ptr<AlgorithmCollectionBuilder> gBuilder;
static std::mutex gBuilderMu;

std::shared_ptr<AlgorithmCollectionBuilder> AlgorithmCollectionBuilder::getInstance() {
  std::lock_guard<std::mutex> lk(gBuilderMu);
  if (!gBuilder) gBuilder = std::shared_ptr<AlgorithmCollectionBuilder>(new AlgorithmCollectionBuilder());
  return gBuilder;
}

void AlgorithmCollectionBuilder::reset() {
  std::lock_guard<std::mutex> lk(gBuilderMu);
  gBuilder.reset();
}

void AlgorithmCollectionBuilder::addAlgorithmBuilder(std::shared_ptr<AlgorithmBuilder> builder) {
  algoBuilders_.push_back(std::move(builder));
}

void AlgorithmCollectionBuilder::setAlgorithmSelector(AlgoSelectFunc selector) { algoSelector_ = std::move(selector); }

void AlgorithmCollectionBuilder::setFallbackAlgorithmSelector(AlgoSelectFunc selector) {
  fallbackAlgoSelector_ = std::move(selector);
}

AlgorithmCollection AlgorithmCollectionBuilder::build() {
  AlgorithmCollection c;
  for (const auto& b : algoBuilders_) {
    auto algo = b->build();
    c.registerAlgorithm(algo->collective(), algo->name(), algo);
  }
  c.setSelectors(algoSelector_, fallbackAlgoSelector_);
  return c;
}

AlgorithmCollection AlgorithmCollectionBuilder::buildDefaultAlgorithms(ncclComm_t comm) {
  if (!comm) throw std::invalid_argument("buildDefaultAlgorithms: null communicator");
  AlgorithmCollection c;
  const size_t kAny = UINT64_MAX;
  struct Def {
    const char* name;
    const char* coll;
    int code, mode;
    size_t lo, hi;
  };
  const Def defs[] = {
      {"default_allreduce_allpair_packet", "allreduce", MSCCLPP_AMD_ALGO_ALLPAIR, 0, 0, kAny},
      {"default_allreduce_packet", "allreduce", MSCCLPP_AMD_ALGO_PACKET, 0, 0, kAny},
      {"default_allreduce_fullmesh", "allreduce", MSCCLPP_AMD_ALGO_FULLMESH, 0, 0, kAny},
      {"default_allreduce_rsag", "allreduce", MSCCLPP_AMD_ALGO_RSAG, 0, 0, kAny},
      {"default_allreduce_rsag_zero_copy", "allreduce", MSCCLPP_AMD_ALGO_RSAG_ZC, 0, 0, kAny},
      {"default_allreduce_rsag_pipeline", "allreduce", MSCCLPP_AMD_ALGO_RSAG_PIPELINE, 0, 0, kAny},
      {"default_allgather_fullmesh2", "allgather", MSCCLPP_AMD_ALGO_FULLMESH, 2, 0, kAny},
      {"default_reducescatter_fullmesh", "reducescatter", MSCCLPP_AMD_ALGO_FULLMESH, 1, 0, kAny},
  };
  for (const auto& d : defs) c.registerAlgorithm(d.coll, d.name, builtin(comm, d.name, d.coll, d.code, d.mode, d.lo, d.hi));
  c.setSelectors(algoSelector_, fallbackAlgoSelector_);
  return c;
}

}  // namespace collective
}  // namespace mscclpp_amd

// ncclCommInitRank's step (nccl.cc:308-314): the fallback selector is the built-in one, the
// collection holds the built-in algorithms extended with the user's.
void ncclComm::buildAlgorithms() {
  using mscclpp_amd::collective::AlgorithmCollectionBuilder;
  cxx = std::make_shared<mscclpp_amd::Communicator>(this);
  auto b = AlgorithmCollectionBuilder::getInstance();
  b->setFallbackAlgorithmSelector(mscclpp_amd::defaultAlgoSelector);
  algos = std::make_unique<mscclpp_amd::AlgorithmCollection>(b->buildDefaultAlgorithms(this));
  algos->extend(b->build());
}
