// Execution plans (JSON) and the executor that runs them over a communicator.
//
// Reference: src/core/executor/execution_plan.cc (plan parsing and lowering: every offset and size
// rule below cites its lines) and src/core/executor/executor.cc (context setup and launch).  The
// setup here is this build's own: one uncached scratch per context mapped into every peer through
// IPC, memory-channel semaphores as [peer][tag] token slots (a channel's tag is its ordinal among
// this rank's channels to that peer, which is how the reference pairs connections,
// executor.cc:286-300), and peer buffer pointers exchanged exactly (so remote offsets need no
// "constant offset" correction, execution_plan.cc:480-493).
#include <fstream>
#include <sstream>

#include "comm_internal.hpp"
#include "executor_common.hpp"
#include "json.hpp"
#include "mscclpp_amd/executor.h"

namespace mscclpp_amd {
int launchExecutionKernel(const exec::TbPlan* plans, int nblocks, int nthreads, size_t ldsBytes, void* input,
                          void* output, void* scratch, uint64_t scratchOffset, uint64_t scratchChunk, uint32_t flag,
                          exec::Syncer* syncers, exec::Sem* sems, int dtype, bool ll16, bool reuseScratch,
                          uint64_t budget, uint32_t* err, hipStream_t s);
}

namespace {

using mscclpp_amd::json::Value;
namespace ex = mscclpp_amd::exec;

constexpr uint64_t kPredefinedScratch = 1ull << 26;       // PREDFINED_SCRATCH_SIZE (execution_common.hpp:20)
constexpr uint64_t kDefaultReuseScratch = 1ull << 27;     // Executor::Impl::defaultScratchBufferSize

struct PlanError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// execution_plan.cc:25-87
uint8_t opTypeOf(const std::string& s) {
  static const std::map<std::string, uint8_t> m = {
      {"nop", ex::NOP},
      {"barrier", ex::BARRIER},
      {"put", ex::PUT},
      {"pws", ex::PUT_WITH_SIGNAL},
      {"pwsf", ex::PUT_WITH_SIGNAL_AND_FLUSH},
      {"get", ex::GET},
      {"copy", ex::COPY},
      {"signal", ex::SIGNAL},
      {"wait", ex::WAIT},
      {"flush", ex::FLUSH},
      {"re", ex::REDUCE},
      {"res", ex::REDUCE_SEND},
      {"rre", ex::READ_REDUCE},
      {"rres", ex::READ_REDUCE_SEND},
      {"ppkt", ex::PUT_PACKETS},
      {"rppkt", ex::READ_PUT_PACKETS},
      {"respkt", ex::REDUCE_SEND_PACKETS},
      {"cpkt", ex::COPY_PACKETS},
      {"upkt", ex::UNPACK_PACKETS},
      {"repkt", ex::REDUCE_PACKETS},
      {"recpkt", ex::REDUCE_COPY_PACKETS},
      {"recspkt", ex::REDUCE_COPY_SEND_PACKETS},
      {"glres", ex::MULTI_LOAD_REDUCE_STORE},
      {"gstore", ex::MULTI_STORE},
      {"gstorepkt", ex::MULTI_STORE_PKT},
      {"rlxsignal", ex::RELAXED_SIGNAL},
      {"rlxwait", ex::RELAXED_WAIT},
      {"pipeline", ex::PIPELINE},
      {"sem_acquire", ex::SEM_ACQUIRE},
      {"sem_release", ex::SEM_RELEASE},
  };
  auto it = m.find(s);
  if (it == m.end()) throw PlanError("invalid operation type: " + s);
  if (it->second == ex::MULTI_LOAD_REDUCE_STORE || it->second == ex::MULTI_STORE || it->second == ex::MULTI_STORE_PKT)
    throw PlanError("operation '" + s + "' needs NVLS multimem, which MI355X does not have");
  return it->second;
}

// execution_plan.cc:89-100
uint8_t bufTypeOf(const std::string& s) {
  if (s == "i") return ex::kInput;
  if (s == "o") return ex::kOutput;
  if (s == "s") return ex::kScratch;
  throw PlanError("invalid buffer type: " + s);
}

enum ChanType { kChanNone, kChanMemory, kChanPort, kChanSwitch };
// execution_plan.cc:102-114
ChanType chanTypeOf(const std::string& s) {
  if (s == "memory") return kChanMemory;
  if (s == "port") return kChanPort;
  if (s == "none") return kChanNone;
  if (s == "switch") return kChanSwitch;
  throw PlanError("invalid channel type: " + s);
}

const char* opName(uint8_t t) {
  static const char* n[] = {"nop",    "barrier", "put",   "ppkt",   "rppkt", "pws",      "pwsf",      "get",
                            "copy",   "cpkt",    "upkt",  "signal", "wait",  "flush",    "re",        "repkt",
                            "recpkt", "res",     "respkt", "recspkt", "rre", "rres",     "glres",     "rlxsignal",
                            "rlxwait", "pipeline", "sem_release", "sem_acquire", "gstore", "gstorepkt"};
  return t < sizeof(n) / sizeof(n[0]) ? n[t] : "?";
}

}  // namespace

struct mscclppAmdExecutionPlan {
  std::string path;
  int rank = 0;
  Value doc;
  std::string name, collective, protocol;
  bool inplace = false, reuse = false, dbl = false, usingPacket = false;
  uint64_t align = 16, minMsg = 0, maxMsg = ~0ull;
  int nthreads = 1024;

  // lowered for one (inputSize, outputSize)
  uint64_t inputSize = 0, outputSize = 0;
  uint64_t inputChunks = 0, outputChunks = 0, scratchChunks = 0;
  struct Chan {
    int peer;
    int tag;
  };
  struct RemoteBuf {
    int peer;
    uint8_t type;
  };
  std::vector<Chan> memChannels;                   // this rank's memory channels, global order
  std::vector<RemoteBuf> remoteBuffers;            // gpu["remote_buffers"] of this rank
  std::vector<std::vector<int>> tbChannels;        // per threadblock: global memory channel index
  std::vector<std::vector<int>> tbRemote;          // per threadblock: global remote buffer id
  std::vector<std::vector<ex::Op>> ops;            // per threadblock
  std::vector<int64_t> semInit;

  mscclppAmdExecutionPlan(const std::string& p, int r) : path(p), rank(r) {
    std::ifstream f(path);
    if (!f) throw PlanError("cannot open plan " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    doc = mscclpp_amd::json::parse(ss.str());
    // ExecutionPlan::Impl::Impl (execution_plan.cc:124-135)
    name = doc["name"].str();
    collective = doc["collective"].str();
    inplace = doc["inplace"].asBool();
    reuse = doc.boolOr("reuse_resources", false);
    dbl = doc.boolOr("use_double_scratch_buffer", false);
    align = doc.u64Or("buffer_alignment", 16);
    minMsg = doc.u64Or("min_message_size", 0);
    maxMsg = doc.u64Or("max_message_size", ~0ull);
    if (align == 0) throw PlanError("buffer_alignment must be positive");
    const Value& gpus = doc["gpus"];
    if (rank < 0 || (size_t)rank >= gpus.size()) throw PlanError("plan has no gpu entry for rank " + std::to_string(rank));
  }

  // calcOffset / calcSize (execution_plan.cc:638-649)
  uint64_t calcOffset(uint64_t size, uint64_t index, uint64_t slices) const {
    const uint64_t nelems = size / align;
    const uint64_t minN = nelems / slices, rem = nelems % slices;
    return (index * minN + std::min<uint64_t>(index, rem)) * align;
  }
  uint64_t calcSize(uint64_t size, uint64_t index, uint64_t slices) const {
    return calcOffset(size, index + 1, slices) - calcOffset(size, index, slices);
  }
  // getSizeAndChunks (execution_plan.cc:610-636)
  std::pair<uint64_t, uint64_t> sizeAndChunks() const {
    if (inputChunks == 0 && outputChunks == 0) throw PlanError("output or input chunks must be greater than 0");
    if (inputChunks && outputChunks) {
      if (inputSize / inputChunks != outputSize / outputChunks) throw PlanError("size per chunk inconsistent");
      return {inputSize, inputChunks};
    }
    if (inputChunks) return {inputSize, inputChunks};
    return {outputSize, outputChunks};
  }
  // calScratchBufferSize / calMaxScratchChunkSize (execution_plan.cc:189-231)
  uint64_t scratchBufferSize(uint64_t in, uint64_t out) const {
    if (reuse && scratchChunks > 0) return kPredefinedScratch;
    uint64_t per = 0;
    if (inputChunks) per = (in + inputChunks - 1) / inputChunks;
    else if (outputChunks) per = (out + outputChunks - 1) / outputChunks;
    else throw PlanError("output or input chunks must be greater than 0");
    uint64_t size = per * scratchChunks * (usingPacket ? 2 : 1);
    if (dbl) size *= 2;
    return (size + align - 1) / align * align;
  }
  uint64_t maxScratchChunk(uint64_t scratchSize) const {
    if (scratchChunks == 0) return 0;
    if (dbl) scratchSize /= 2;
    uint64_t size = (scratchSize + scratchChunks - 1) / scratchChunks;
    return (size + align - 1) / align * align;
  }
  // getOffset / getBufferSize (execution_plan.cc:651-672)
  uint64_t chunkOffset(uint64_t chunk, uint8_t type) const {
    auto [size, n] = sizeAndChunks();
    const uint64_t chunkSize = (size + n - 1) / n;
    const uint64_t scr = maxScratchChunk(kPredefinedScratch);
    if (type == ex::kScratch && reuse && scr < chunkSize) return chunk * maxScratchChunk(kPredefinedScratch);
    return calcOffset(size, chunk, n);
  }
  uint64_t chunkBytes(uint64_t index, uint64_t nChunks) const {
    return chunkOffset(index + nChunks, ex::kNoBuffer) - chunkOffset(index, ex::kNoBuffer);
  }
  uint64_t upperBoundChunk() const {  // getUpperBoundChunkSize (:674-687)
    if (inputChunks) return (inputSize / align + inputChunks - 1) / inputChunks * align;
    if (outputChunks) return (outputSize / align + outputChunks - 1) / outputChunks * align;
    throw PlanError("output or input chunks must be greater than 0");
  }

  // loadExecutionPlan (execution_plan.cc:233-267) for one message size
  void load(uint64_t in, uint64_t out) {
    usingPacket = doc["protocol"].str() == "LL";
    inputSize = in;
    outputSize = out;
    nthreads = (int)doc.u64Or("num_threads_per_block", 1024);
    const Value& gpus = doc["gpus"];
    const Value& gpu = gpus[(size_t)rank];
    if ((int)gpu["id"].asI64() != rank) throw PlanError("GPU rank does not match");
    inputChunks = gpu["input_chunks"].asU64();
    outputChunks = gpu["output_chunks"].asU64();
    scratchChunks = gpu["scratch_chunks"].asU64();
    checkMessageSize();
    setupChannels(gpu);
    setupRemoteBuffers(gpu);
    semInit.clear();
    if (gpu.contains("semaphores"))
      for (auto& s : gpu["semaphores"].arr) semInit.push_back(s["init_value"].asI64());
    if (semInit.size() > (size_t)ex::kMaxSemaphores) throw PlanError("too many semaphores");
    setupOperations(gpu);
  }

  // checkMessageSize (execution_plan.cc:297-311)
  void checkMessageSize() const {
    if (inputSize % align || outputSize % align || (inputChunks && (inputSize / align) % inputChunks) ||
        (outputChunks && (outputSize / align) % outputChunks))
      throw PlanError("input or output size is not aligned with buffer alignment or chunks");
    const uint64_t size = collective == "allgather" ? outputSize : inputSize;
    if (size < minMsg || size > maxMsg) throw PlanError("input or output size is not within the valid range");
  }

  // parseChannels / setupChannels (execution_plan.cc:313-399)
  void setupChannels(const Value& gpu) {
    memChannels.clear();
    std::map<int, int> tagOf;
    for (auto& ch : gpu["channels"].arr) {
      ChanType t = chanTypeOf(ch["channel_type"].str());
      if (t == kChanSwitch) throw PlanError("switch (NVLS) channels do not exist on MI355X");
      if (t == kChanPort)
        throw PlanError("port channels are not supported by this executor: one-node plans use memory channels");
      for (auto& p : ch["connected_to"].arr) {
        const int peer = (int)p.asI64();
        if (peer < 0 || peer >= ex::kMaxRanks || peer == rank) throw PlanError("bad connected_to peer");
        const int tag = tagOf[peer]++;
        if (tag >= ex::kMaxTags) throw PlanError("too many channels to one peer");
        memChannels.push_back({peer, tag});
      }
    }
    tbChannels.assign(gpu["threadblocks"].size(), {});
    for (auto& tb : gpu["threadblocks"].arr) {
      const size_t id = tb["id"].asU64();
      if (id >= tbChannels.size()) throw PlanError("threadblock id out of range");
      if (!tb.contains("channels")) continue;
      for (auto& ch : tb["channels"].arr) {
        ChanType t = chanTypeOf(ch["channel_type"].str());
        if (t != kChanMemory) throw PlanError("only memory channels are supported in threadblocks");
        for (auto& cid : ch["channel_ids"].arr) {
          const uint64_t c = cid.asU64();
          if (c >= memChannels.size()) throw PlanError("channel id out of range");
          tbChannels[id].push_back((int)c);
        }
      }
      if (tbChannels[id].size() > (size_t)ex::kMaxChannels) throw PlanError("too many channels in a threadblock");
    }
  }

  // parseRemoteBuffer / setupRemoteBuffers (execution_plan.cc:352-420)
  void setupRemoteBuffers(const Value& gpu) {
    remoteBuffers.clear();
    for (auto& rb : gpu["remote_buffers"].arr) {
      for (auto& a : rb["access_channel_types"].arr)
        if (chanTypeOf(a.str()) != kChanMemory) throw PlanError("remote buffers must be accessed through memory channels");
      remoteBuffers.push_back({(int)rb["rank"].asI64(), bufTypeOf(rb["type"].str())});
    }
    tbRemote.assign(gpu["threadblocks"].size(), {});
    for (auto& tb : gpu["threadblocks"].arr) {
      const size_t id = tb["id"].asU64();
      if (!tb.contains("remote_buffer_refs")) continue;
      for (auto& ref : tb["remote_buffer_refs"].arr) {
        if (chanTypeOf(ref["access_channel_type"].str()) != kChanMemory) throw PlanError("only memory access supported");
        for (auto& b : ref["remote_buffer_ids"].arr) {
          const uint64_t bid = b.asU64();
          if (bid >= remoteBuffers.size()) throw PlanError("remote buffer id out of range");
          tbRemote[id].push_back((int)bid);
        }
      }
      if (tbRemote[id].size() > (size_t)ex::kMaxChannels) throw PlanError("too many remote buffers in a threadblock");
    }
  }

  // setupOperations / setupOperation (execution_plan.cc:436-605)
  void setupOperations(const Value& gpu) {
    ops.assign(gpu["threadblocks"].size(), {});
    for (auto& tb : gpu["threadblocks"].arr) {
      const size_t id = tb["id"].asU64();
      for (auto& o : tb["ops"].arr) {
        ops[id].push_back(lowerOp(o, id));
        if (ops[id].back().type == ex::PIPELINE)
          for (auto& inner : o["ops"].arr) ops[id].push_back(lowerOp(inner, id));
      }
      if (ops[id].size() > (size_t)ex::kMaxOps) throw PlanError("too many operations in a threadblock");
    }
  }

  ex::Op lowerOp(const Value& o, size_t tb) const {
    ex::Op op{};
    op.type = opTypeOf(o["name"].str());
    ChanType ct = kChanNone;
    if (o.contains("channel_type")) {
      ct = chanTypeOf(o["channel_type"].str());
      if (ct == kChanPort || ct == kChanSwitch) throw PlanError("only memory channels are supported");
    }
    if (o.contains("reduce_op")) {
      const std::string r = o["reduce_op"].str();
      if (r == "min") op.reduceOp = 1;
      else if (r != "sum") throw PlanError("unsupported reduce_op " + r);
    }
    if (o.contains("channel_ids")) {
      const auto& ids = o["channel_ids"].arr;
      if (ids.size() > (size_t)ex::kMaxChannelsPerOp) throw PlanError("too many channels in an operation");
      op.nChannels = (uint8_t)ids.size();
      for (size_t i = 0; i < ids.size(); ++i) {
        const uint64_t c = ids[i].asU64();
        if (c >= tbChannels[tb].size()) throw PlanError("operation channel id out of range");
        op.chan[i] = (uint8_t)c;
      }
    }
    uint64_t tbId = 0, tbgSize = 1;
    if (o.contains("tbg_info")) {
      tbId = o["tbg_info"]["tb_id"].asU64();
      tbgSize = o["tbg_info"]["tbg_size"].asU64();
      if (tbgSize == 0 || tbId >= tbgSize) throw PlanError("bad tbg_info");
    }
    auto lowerBuffers = [&](const char* key, uint8_t& n, uint8_t* refs, uint64_t* offs, uint64_t* sizes) {
      if (!o.contains(key)) return;
      const auto& list = o[key].arr;
      if (list.size() > (size_t)ex::kMaxBuffersPerOp) throw PlanError("too many buffers in an operation");
      n = (uint8_t)list.size();
      for (size_t i = 0; i < list.size(); ++i) {
        const Value& b = list[i];
        uint8_t type = ex::kNoBuffer;
        refs[i] = ex::kNoBuffer;
        if (b.contains("type")) {
          type = bufTypeOf(b["type"].str());
          refs[i] = type;
        }
        if (b.contains("buffer_id")) {
          const uint64_t j = b["buffer_id"].asU64();  // threadblock-local remote buffer index
          if (j >= tbRemote[tb].size()) throw PlanError("operation buffer_id out of range");
          refs[i] = (uint8_t)j;
          type = remoteBuffers[tbRemote[tb][j]].type;
        }
        if (b.contains("switch_channel_id")) throw PlanError("switch channels do not exist on MI355X");
        uint64_t off = chunkOffset(b["index"].asU64(), type);
        uint64_t size = chunkBytes(b["index"].asU64(), b["size"].asU64());
        off += calcOffset(size, tbId, tbgSize);
        size = calcSize(size, tbId, tbgSize);
        offs[i] = off;
        sizes[i] = size;
      }
    };
    lowerBuffers("src_buff", op.nInputs, op.inRef, op.inOff, op.inSize);
    lowerBuffers("dst_buff", op.nOutputs, op.outRef, op.outOff, op.outSize);
    if (o.contains("barrier_id")) op.syncer = (uint32_t)o["barrier_id"].asU64();
    if (o.contains("num_threadblocks")) op.nThreadBlocks = (uint32_t)o["num_threadblocks"].asU64();
    if (op.type == ex::BARRIER && op.syncer >= (uint32_t)ex::kMaxSyncers) throw PlanError("barrier id out of range");
    if (o.contains("semaphore_ids")) {
      const auto& ids = o["semaphore_ids"].arr;
      if (ids.size() > (size_t)ex::kMaxSemaphores) throw PlanError("too many semaphores in an operation");
      op.nSems = (uint8_t)ids.size();
      for (size_t i = 0; i < ids.size(); ++i) {
        const uint64_t s = ids[i].asU64();
        if (s >= (uint64_t)ex::kMaxSemaphores) throw PlanError("semaphore id out of range");
        op.semIds[i] = (uint8_t)s;
      }
    }
    if (o.contains("iter_context")) {
      op.unitSize = o["iter_context"]["unit_size"].asU64();
      if (op.unitSize == 0) throw PlanError("pipeline unit_size must be positive");
      op.nOperations = (uint32_t)o["ops"].size();
      const uint64_t nChunks = o["iter_context"]["num_chunks"].asU64();
      const uint64_t sizes = nChunks * upperBoundChunk();
      op.nIterations = (uint32_t)((sizes + op.unitSize - 1) / op.unitSize);
    }
    return op;
  }

  std::string describe() const {
    std::ostringstream s;
    s << "{\"name\":\"" << name << "\",\"rank\":" << rank << ",\"nthreads\":" << nthreads
      << ",\"packet\":" << (usingPacket ? "true" : "false") << ",\"channels\":[";
    for (size_t i = 0; i < memChannels.size(); ++i)
      s << (i ? "," : "") << "[" << memChannels[i].peer << "," << memChannels[i].tag << "]";
    s << "],\"remote_buffers\":[";
    for (size_t i = 0; i < remoteBuffers.size(); ++i)
      s << (i ? "," : "") << "[" << remoteBuffers[i].peer << "," << (int)remoteBuffers[i].type << "]";
    s << "],\"threadblocks\":[";
    for (size_t t = 0; t < ops.size(); ++t) {
      s << (t ? "," : "") << "{\"channels\":[";
      for (size_t i = 0; i < tbChannels[t].size(); ++i) s << (i ? "," : "") << tbChannels[t][i];
      s << "],\"remote\":[";
      for (size_t i = 0; i < tbRemote[t].size(); ++i) s << (i ? "," : "") << tbRemote[t][i];
      s << "],\"ops\":[";
      for (size_t k = 0; k < ops[t].size(); ++k) {
        const ex::Op& op = ops[t][k];
        s << (k ? "," : "") << "{\"op\":\"" << opName(op.type) << "\",\"reduce\":" << (int)op.reduceOp << ",\"chan\":[";
        for (int i = 0; i < op.nChannels; ++i) s << (i ? "," : "") << (int)op.chan[i];
        s << "],\"in\":[";
        for (int i = 0; i < op.nInputs; ++i)
          s << (i ? "," : "") << "[" << (int)op.inRef[i] << "," << op.inOff[i] << "," << op.inSize[i] << "]";
        s << "],\"out\":[";
        for (int i = 0; i < op.nOutputs; ++i)
          s << (i ? "," : "") << "[" << (int)op.outRef[i] << "," << op.outOff[i] << "," << op.outSize[i] << "]";
        s << "],\"barrier\":[" << op.syncer << "," << op.nThreadBlocks << "],\"sems\":[";
        for (int i = 0; i < op.nSems; ++i) s << (i ? "," : "") << (int)op.semIds[i];
        s << "],\"pipeline\":[" << op.nIterations << "," << op.nOperations << "," << op.unitSize << "]}";
      }
      s << "]}";
    }
    s << "]}";
    return s.str();
  }
};

struct mscclppAmdExecutor {
  ncclComm* comm = nullptr;
  uint64_t* tokens = nullptr;    // inbound [kMaxRanks][kMaxTags], uncached
  uint64_t* expected = nullptr;  // [kMaxRanks][kMaxTags]
  PeerBufs peerTokens;
  ex::Syncer* syncers = nullptr;
  uint32_t* err = nullptr;
  uint32_t flag = 0;  // Executor::Impl::launchKernel's flag: +1 per execution

  struct DevicePlan {
    ex::TbPlan* dev = nullptr;
    int nblocks = 0;
    size_t lds = 0;
  };
  struct Context {
    void* scratch = nullptr;
    uint64_t scratchBytes = 0, scratchChunk = 0;
    PeerBufs peerScratch, peerIn, peerOut;
    ex::Sem* sems = nullptr;
    std::map<std::pair<uint64_t, uint64_t>, DevicePlan> plans;
  };
  std::map<std::tuple<uint64_t, uint64_t, std::string>, Context> contexts;

  explicit mscclppAmdExecutor(ncclComm* c) : comm(c) {
    const size_t tokBytes = sizeof(uint64_t) * ex::kMaxRanks * ex::kMaxTags;
    tokens = (uint64_t*)allocUncached(tokBytes);
    HIPCHECK(hipMalloc((void**)&expected, tokBytes));
    memsetSync(expected, 0, tokBytes);
    HIPCHECK(hipMalloc((void**)&syncers, sizeof(ex::Syncer) * ex::kMaxSyncers));
    memsetSync(syncers, 0, sizeof(ex::Syncer) * ex::kMaxSyncers);
    HIPCHECK(hipMalloc((void**)&err, 256));
    memsetSync(err, 0, 256);
    HIPCHECK(hipDeviceSynchronize());
    if (comm->nranks > 1) peerTokens = comm->exchange(tokens);
    else peerTokens[0] = tokens;
    comm->boot->barrier();
  }

  void dropContexts() {
    HIPCHECK(hipDeviceSynchronize());
    comm->boot->barrier();  // no rank still runs a kernel on these buffers
    for (auto& kv : contexts) {
      Context& c = kv.second;
      c.peerScratch = c.peerIn = c.peerOut = PeerBufs();  // our mappings of the peers' buffers close
    }
    comm->boot->barrier();  // every rank closed its mappings of our scratch before it is freed
    for (auto& kv : contexts) {
      Context& c = kv.second;
      if (c.scratch) freeDevice(c.scratch);
      if (c.sems) freeDevice(c.sems);
      for (auto& p : c.plans) freeDevice(p.second.dev);
    }
    contexts.clear();
  }

  void destroy() {
    dropContexts();
    peerTokens = PeerBufs();
    comm->boot->barrier();
    freeDevice(tokens);
    freeDevice(expected);
    freeDevice(syncers);
    freeDevice(err);
  }

  Context& context(mscclppAmdExecutionPlan& plan, void* send, void* recv, uint64_t sendBytes, uint64_t recvBytes) {
    auto key = std::make_tuple((uint64_t)send, (uint64_t)recv, plan.name);
    auto it = contexts.find(key);
    if (it != contexts.end()) return it->second;
    // setupExecutionContext (executor.cc:145-200): scratch sized from the buffers' allocations
    void* base = nullptr;
    size_t sendRange = 0, recvRange = 0;
    HIPCHECK(hipMemGetAddressRange((hipDeviceptr_t*)&base, &sendRange, (hipDeviceptr_t)send));
    HIPCHECK(hipMemGetAddressRange((hipDeviceptr_t*)&base, &recvRange, (hipDeviceptr_t)recv));
    (void)sendBytes;
    (void)recvBytes;
    Context c;
    // setupScratchBuffer (executor.cc:240-262)
    uint64_t sb = plan.scratchBufferSize(std::min<uint64_t>(sendRange, plan.maxMsg), std::min<uint64_t>(recvRange, plan.maxMsg));
    c.scratchChunk = plan.maxScratchChunk(sb);
    if (plan.reuse) {
      if (sb > kDefaultReuseScratch) throw PlanError("scratch exceeds the default reuse buffer size");
      sb = kDefaultReuseScratch;
    }
    c.scratchBytes = sb;
    c.scratch = allocUncached(std::max<uint64_t>(sb, 256));
    // semaphores (executor.cc:434-443)
    const size_t nsem = std::max<size_t>(plan.semInit.size(), 1);
    std::vector<ex::Sem> sems(nsem);
    for (size_t i = 0; i < plan.semInit.size(); ++i) sems[i].value = plan.semInit[i];
    HIPCHECK(hipMalloc((void**)&c.sems, nsem * sizeof(ex::Sem)));
    HIPCHECK(hipMemcpy(c.sems, sems.data(), nsem * sizeof(ex::Sem), hipMemcpyHostToDevice));
    HIPCHECK(hipDeviceSynchronize());
    // peer pointers (setupRegisteredMemories, executor.cc:314-344): every rank maps every other
    // rank's scratch, input and output exactly
    if (comm->nranks > 1) {
      c.peerScratch = comm->exchange(c.scratch);
      c.peerIn = comm->exchange(send);
      c.peerOut = recv == send ? c.peerIn : comm->exchange(recv);
    } else {
      c.peerScratch[0] = c.scratch;
      c.peerIn[0] = send;
      c.peerOut[0] = recv;
    }
    comm->boot->barrier();
    return contexts.emplace(key, std::move(c)).first->second;
  }

  DevicePlan& devicePlan(Context& c, mscclppAmdExecutionPlan& plan, uint64_t sendBytes, uint64_t recvBytes) {
    auto key = std::make_pair(sendBytes, recvBytes);
    auto it = c.plans.find(key);
    if (it != c.plans.end()) return it->second;
    // setupDeviceExecutionPlan (executor.cc:445-490)
    std::vector<ex::TbPlan> tbs(plan.ops.size());
    size_t maxOps = 0;
    for (size_t t = 0; t < plan.ops.size(); ++t) {
      ex::TbPlan& p = tbs[t];
      std::memset(&p, 0, sizeof(p));
      p.h.nOps = (uint32_t)plan.ops[t].size();
      maxOps = std::max(maxOps, plan.ops[t].size());
      p.h.nChannels = (uint32_t)plan.tbChannels[t].size();
      for (size_t j = 0; j < plan.tbChannels[t].size(); ++j) {
        const auto& ch = plan.memChannels[plan.tbChannels[t][j]];
        const size_t mySlot = (size_t)comm->rank * ex::kMaxTags + ch.tag;
        const size_t peerSlot = (size_t)ch.peer * ex::kMaxTags + ch.tag;
        if (ch.peer >= comm->nranks) throw PlanError("plan channel to a rank outside the communicator");
        p.h.ch[j].remoteToken = (uint64_t*)peerTokens[ch.peer] + mySlot;
        p.h.ch[j].inbound = tokens + peerSlot;
        p.h.ch[j].expected = expected + peerSlot;
      }
      p.h.nRemote = (uint32_t)plan.tbRemote[t].size();
      for (size_t j = 0; j < plan.tbRemote[t].size(); ++j) {
        const auto& rb = plan.remoteBuffers[plan.tbRemote[t][j]];
        if (rb.peer < 0 || rb.peer >= comm->nranks) throw PlanError("remote buffer on a rank outside the communicator");
        p.h.remoteType[j] = rb.type;
        p.h.remotePtr[j] = rb.type == ex::kInput ? c.peerIn[rb.peer]
                           : rb.type == ex::kOutput ? c.peerOut[rb.peer]
                                                    : c.peerScratch[rb.peer];
      }
      for (size_t k = 0; k < plan.ops[t].size(); ++k) p.ops[k] = plan.ops[t][k];
    }
    DevicePlan d;
    d.nblocks = (int)tbs.size();
    d.lds = sizeof(ex::TbHeader) + maxOps * sizeof(ex::Op);
    d.lds = (d.lds + 15) / 16 * 16;
    HIPCHECK(hipMalloc((void**)&d.dev, sizeof(ex::TbPlan) * std::max<size_t>(tbs.size(), 1)));
    HIPCHECK(hipMemcpy(d.dev, tbs.data(), sizeof(ex::TbPlan) * tbs.size(), hipMemcpyHostToDevice));
    return c.plans.emplace(key, d).first->second;
  }

  int execute(int rank, void* send, void* recv, uint64_t sendBytes, uint64_t recvBytes, int dtype,
              mscclppAmdExecutionPlan& plan, hipStream_t stream, int packetType) {
    if (rank != comm->rank || rank != plan.rank) throw PlanError("rank does not match the communicator / plan");
    int dt = -1;
    switch (dtype) {
      case MSCCLPP_AMD_DT_INT32: dt = MSCCLPP_AMD_I32; break;
      case MSCCLPP_AMD_DT_UINT32: dt = MSCCLPP_AMD_U32; break;
      case MSCCLPP_AMD_DT_FLOAT16: dt = MSCCLPP_AMD_F16; break;
      case MSCCLPP_AMD_DT_FLOAT32: dt = MSCCLPP_AMD_F32; break;
      case MSCCLPP_AMD_DT_BFLOAT16: dt = MSCCLPP_AMD_BF16; break;
      // the FP8 kernels of execution_kernel.hpp:949-1000 (T == AccumT); gfx950 converts the OCP
      // formats in hardware and, like the reference on a platform without the other variant
      // (:952-960, :975-983), rejects FNUZ
      case MSCCLPP_AMD_DT_FLOAT8_E4M3FN: dt = MSCCLPP_AMD_E4M3; break;
      case MSCCLPP_AMD_DT_FLOAT8_E5M2: dt = MSCCLPP_AMD_E5M2; break;
      case MSCCLPP_AMD_DT_FLOAT8_E4M3B15: dt = MSCCLPP_AMD_E4M3B15; break;  // execution_kernel.hpp:997-1007
      case MSCCLPP_AMD_DT_UINT8: dt = MSCCLPP_AMD_U8; break;                 // :1008-1018
      case MSCCLPP_AMD_DT_FLOAT8_E4M3FNUZ:
      case MSCCLPP_AMD_DT_FLOAT8_E5M2FNUZ:
        warn("execution plan: FNUZ fp8 is not natively supported on gfx950; use the OCP FLOAT8_E4M3FN / FLOAT8_E5M2");
        return ncclInvalidUsage;
      default: return ncclInvalidArgument;
    }
    if (packetType != MSCCLPP_AMD_PACKET_LL8 && packetType != MSCCLPP_AMD_PACKET_LL16) return ncclInvalidArgument;
    if ((int)plan.doc["gpus"].size() != comm->nranks) throw PlanError("plan rank count differs from the communicator");
    if (plan.inputSize != sendBytes || plan.outputSize != recvBytes || plan.ops.empty()) plan.load(sendBytes, recvBytes);
    Context& c = context(plan, send, recv, sendBytes, recvBytes);
    DevicePlan& d = devicePlan(c, plan, sendBytes, recvBytes);
    // launchKernelHelper (executor.cc:492-513)
    ++flag;
    const uint64_t scrOff = (plan.dbl && (flag & 1u) == 0) ? c.scratchBytes / 2 : 0;
    const int rc = launchExecutionKernel(d.dev, d.nblocks, plan.nthreads, d.lds, send, recv, c.scratch, scrOff,
                                         c.scratchChunk, flag, syncers, c.sems, dt, packetType == MSCCLPP_AMD_PACKET_LL16,
                                         plan.reuse, spinBudgetTicks(), err, stream);
    if (rc == 5) warn("execution plan grid (" + std::to_string(d.nblocks) + " x " + std::to_string(plan.nthreads) +
                      ") cannot be resident at once on this device");
    return rc == 0 ? ncclSuccess : rc == 1 ? ncclUnhandledCudaError : rc == 4 ? ncclInvalidArgument : ncclInvalidUsage;
  }
};

// =============================================================================================
// C ABI
// =============================================================================================
namespace {
template <typename F>
int planGuarded(F&& f) {
  return guarded([&] {
    try {
      return f();
    } catch (const PlanError& e) {
      warn(std::string("execution plan: ") + e.what());
      return (int)ncclInvalidArgument;
    } catch (const std::runtime_error& e) {  // json errors
      if (dynamic_cast<const HipError*>(&e)) throw;
      warn(std::string("execution plan: ") + e.what());
      return (int)ncclInvalidArgument;
    }
  });
}
}  // namespace

extern "C" {

int mscclppAmdExecutionPlanCreate(const char* planPath, int rank, mscclppAmdExecutionPlan_t* plan) {
  return planGuarded([&] {
    if (!planPath || !plan) return (int)ncclInvalidArgument;
    *plan = new mscclppAmdExecutionPlan(planPath, rank);
    return (int)ncclSuccess;
  });
}

int mscclppAmdExecutionPlanDestroy(mscclppAmdExecutionPlan_t plan) {
  delete plan;
  return ncclSuccess;
}

const char* mscclppAmdExecutionPlanName(mscclppAmdExecutionPlan_t plan) { return plan ? plan->name.c_str() : ""; }
const char* mscclppAmdExecutionPlanCollective(mscclppAmdExecutionPlan_t plan) {
  return plan ? plan->collective.c_str() : "";
}
size_t mscclppAmdExecutionPlanMinMessageSize(mscclppAmdExecutionPlan_t plan) { return plan ? plan->minMsg : 0; }
size_t mscclppAmdExecutionPlanMaxMessageSize(mscclppAmdExecutionPlan_t plan) { return plan ? plan->maxMsg : 0; }
int mscclppAmdExecutionPlanIsInPlace(mscclppAmdExecutionPlan_t plan) { return plan && plan->inplace ? 1 : 0; }

int mscclppAmdExecutionPlanDescribe(mscclppAmdExecutionPlan_t plan, size_t inputBytes, size_t outputBytes, char* buf,
                                    size_t len, size_t* needed) {
  return planGuarded([&] {
    if (!plan) return (int)ncclInvalidArgument;
    plan->load(inputBytes, outputBytes);
    const std::string s = plan->describe();
    if (needed) *needed = s.size() + 1;
    if (buf && len) {
      const size_t n = std::min(len - 1, s.size());
      std::memcpy(buf, s.data(), n);
      buf[n] = 0;
    }
    return (int)ncclSuccess;
  });
}

int mscclppAmdExecutorCreate(ncclComm_t comm, mscclppAmdExecutor_t* executor) {
  return guarded([&] {
    if (!comm || !executor) return (int)ncclInvalidArgument;
    *executor = new mscclppAmdExecutor(comm);
    return (int)ncclSuccess;
  });
}

int mscclppAmdExecutorExecute(mscclppAmdExecutor_t executor, int rank, void* sendbuff, void* recvbuff, size_t sendBytes,
                              size_t recvBytes, int dtype, mscclppAmdExecutionPlan_t plan, void* stream,
                              int packetType) {
  return planGuarded([&] {
    if (!executor || !plan || !sendbuff || !recvbuff) return (int)ncclInvalidArgument;
    std::lock_guard<std::mutex> lk(executor->comm->mu);
    return executor->execute(rank, sendbuff, recvbuff, sendBytes, recvBytes, dtype, *plan, (hipStream_t)stream,
                             packetType);
  });
}

int mscclppAmdExecutorReset(mscclppAmdExecutor_t executor) {
  return guarded([&] {
    if (!executor) return (int)ncclInvalidArgument;
    std::lock_guard<std::mutex> lk(executor->comm->mu);
    executor->dropContexts();
    return (int)ncclSuccess;
  });
}

int mscclppAmdExecutorDestroy(mscclppAmdExecutor_t executor) {
  return guarded([&] {
    if (!executor) return (int)ncclInvalidArgument;
    {
      std::lock_guard<std::mutex> lk(executor->comm->mu);
      executor->destroy();
    }
    delete executor;
    return (int)ncclSuccess;
  });
}

int mscclppAmdExecutorGetDeviceError(mscclppAmdExecutor_t executor, uint32_t* words4, int clear) {
  return guarded([&] {
    if (!executor || !words4) return (int)ncclInvalidArgument;
    HIPCHECK(hipDeviceSynchronize());
    HIPCHECK(hipMemcpy(words4, executor->err, 16, hipMemcpyDeviceToHost));
    if (clear) memsetSync(executor->err, 0, 16);
    return (int)ncclSuccess;
  });
}

}  // extern "C"
