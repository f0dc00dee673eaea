// The C++ algorithm plugin interface (include/mscclpp_amd/algorithm.hpp), exercised the way the
// reference's examples/customized-collective-algorithm/customized_allgather.cu uses
// mscclpp::AlgorithmCollectionBuilder: a user algorithm builder and selector registered before
// ncclCommInitRank, then reached through ncclAllGather / ncclAllReduce.
//
//   test_algorithm_plugin cpu        host-only checks (no GPU touched)
//   test_algorithm_plugin gpu <n>    n forked processes, one rank each (rank % device count)
#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <cmath>
#include <memory>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "mscclpp_amd/algorithm.hpp"
#include "mscclpp_amd/nccl.h"

using namespace mscclpp_amd;

#define CHECK(cond)                                                               \
  do {                                                                            \
    if (!(cond)) {                                                                \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)
#define HIP_OK(cmd) CHECK((cmd) == hipSuccess)
#define NCCL_OK(cmd) CHECK((cmd) == ncclSuccess)

static const std::unordered_map<std::string, std::vector<uint64_t>> kNoHints;

// A host-only algorithm whose kernel records what it was called with.
struct Probe {
  int inits = 0, ctxs = 0, calls = 0;
  DataType lastAccum = DataType::AUTO;
};

static std::shared_ptr<NativeAlgorithm> probeAlgo(const std::string& name, const std::string& coll, Probe* p) {
  return std::make_shared<NativeAlgorithm>(
      name, coll, [p](std::shared_ptr<Communicator>) { p->inits++; },
      [p](const std::shared_ptr<void> ctx, const void*, void*, size_t, size_t, DataType, ReduceOp, hipStream_t, int,
          int, const std::unordered_map<std::string, uintptr_t>&, DataType accum) {
        CHECK(*std::static_pointer_cast<int>(ctx) == 7);
        p->calls++;
        p->lastAccum = accum;
        return CommResult::CommSuccess;
      },
      [p](std::shared_ptr<Communicator>, const void*, void*, size_t, size_t, DataType) {
        p->ctxs++;
        return std::static_pointer_cast<void>(std::make_shared<int>(7));
      },
      [](const void* in, void* out, size_t is, size_t os, DataType, bool) {
        return AlgorithmCtxKey{const_cast<void*>(in), out, is, os, 0};
      });
}

static int runCpu() {
  // NativeAlgorithm: init once, one context per key, accumDtype AUTO -> dtype (algorithm.cc:42-68)
  Probe p;
  auto a = probeAlgo("probe", "allreduce", &p);
  char b1[64], b2[64];
  for (int i = 0; i < 3; ++i)
    CHECK(a->execute(nullptr, b1, b1, 64, 64, DataType::FLOAT16, SUM, nullptr, nullptr) == CommResult::CommSuccess);
  CHECK(p.inits == 1 && p.ctxs == 1 && p.calls == 3 && p.lastAccum == DataType::FLOAT16);
  a->execute(nullptr, b2, b2, 64, 64, DataType::FLOAT8_E4M3FN, SUM, nullptr, nullptr, 0, 0, false, {},
             DataType::FLOAT32);
  CHECK(p.inits == 1 && p.ctxs == 2 && a->numContexts() == 2 && p.lastAccum == DataType::FLOAT32);
  a->reset();
  CHECK(a->numContexts() == 0);
  a->execute(nullptr, b1, b1, 64, 64, DataType::FLOAT16, SUM, nullptr, nullptr);
  CHECK(p.inits == 1 && p.ctxs == 3);
  CHECK(a->messageRange().first == 0 && a->messageRange().second == UINT64_MAX);
  a->setMessageSizeRange(16, 1024);
  CHECK(a->messageRange().first == 16 && a->messageRange().second == 1024);
  CHECK(a->type() == AlgorithmType::Native && a->bufferMode() == CollectiveBufferMode::Any);

  // CollectiveRequest::bufferMode (algorithm.cc:13-24)
  const std::string ar("allreduce"), ag("allgather");
  char buf[4096];
  CollectiveRequest inplace{8, 8, 3, buf, buf, 256, nullptr, ar, DataType::FLOAT16, kNoHints};
  CollectiveRequest oop{8, 8, 3, buf, buf + 2048, 256, nullptr, ar, DataType::FLOAT16, kNoHints};
  CollectiveRequest agIn{8, 8, 3, buf + 3 * 256, buf, 256, nullptr, ag, DataType::FLOAT16, kNoHints};
  CollectiveRequest agOut{8, 8, 3, buf + 2 * 256, buf, 256, nullptr, ag, DataType::FLOAT16, kNoHints};
  CHECK(inplace.bufferMode() == CollectiveBufferMode::InPlace);
  CHECK(oop.bufferMode() == CollectiveBufferMode::OutOfPlace);
  CHECK(agIn.bufferMode() == CollectiveBufferMode::InPlace);
  CHECK(agOut.bufferMode() == CollectiveBufferMode::OutOfPlace);

  // AlgorithmCollection: no selector -> invalid usage; primary then fallback (algorithm.cc:98-110)
  AlgorithmCollection c;
  Probe q;
  c.registerAlgorithm("allreduce", "default_allreduce_allpair_packet", probeAlgo("default_allreduce_allpair_packet", "allreduce", &q));
  c.registerAlgorithm("allreduce", "default_allreduce_packet", probeAlgo("default_allreduce_packet", "allreduce", &q));
  c.registerAlgorithm("allreduce", "default_allreduce_fullmesh", probeAlgo("default_allreduce_fullmesh", "allreduce", &q));
  c.registerAlgorithm("allgather", "default_allgather_fullmesh2", probeAlgo("default_allgather_fullmesh2", "allgather", &q));
  bool threw = false;
  try {
    c.selectAlgorithm(oop);
  } catch (const std::logic_error&) {
    threw = true;
  }
  CHECK(threw);
  c.setSelectors(nullptr, defaultAlgoSelector);
  auto pick = [&](size_t bytes, const std::string& coll) {
    CollectiveRequest r{8, 8, 0, buf, buf + 1, bytes, nullptr, coll, DataType::FLOAT16, kNoHints};
    auto s = c.selectAlgorithm(r);
    return s ? s->name() : std::string("null");
  };
  // MSCCLPP_AMD_ALGO is read once per process (the reference reads its environment once): the test
  // runs this program with it unset and with MSCCLPP_AMD_ALGO=packet
  const char* forced = std::getenv("MSCCLPP_AMD_ALGO");
  if (forced && std::string(forced) == "packet") {
    CHECK(pick(1024, ar) == "default_allreduce_packet");
    CHECK(pick(48 << 20, ar) == "default_allreduce_packet");
    std::printf("forced OK\n");
    return 0;
  }
  // algorithm_selector.cc:107-131 (AMD): <=16 KiB allpair, <=1 MiB packet, larger fullmesh
  CHECK(pick(1024, ar) == "default_allreduce_allpair_packet");
  CHECK(pick(1 << 14, ar) == "default_allreduce_allpair_packet");
  CHECK(pick((1 << 14) + 2, ar) == "default_allreduce_packet");
  CHECK(pick(1 << 20, ar) == "default_allreduce_packet");
  CHECK(pick(48 << 20, ar) == "default_allreduce_fullmesh");
  CHECK(pick(1 << 20, ag) == "default_allgather_fullmesh2");
  CHECK(pick(1 << 20, "broadcast") == "null");
  Probe u;
  c.registerAlgorithm("allreduce", "mine", probeAlgo("mine", "allreduce", &u));
  c.setSelectors(
      [](const AlgoMapByCollective& m, const CollectiveRequest& r) -> std::shared_ptr<Algorithm> {
        if (r.collective == "allreduce" && r.messageSize == 4096) return m.at("allreduce").at("mine");
        return nullptr;
      },
      defaultAlgoSelector);
  CHECK(pick(4096, ar) == "mine");
  CHECK(pick(8192, ar) == "default_allreduce_allpair_packet");
  CHECK(c.getAlgorithmsByCollective("allreduce").size() == 4);
  CHECK(c.getAlgorithmsByCollective("nope").empty());
  CHECK(c.getAllAlgorithms().size() == 5);
  AlgorithmCollection d;
  d.extend(c);
  CHECK(d.getAllAlgorithms().size() == 5);

  // AlgorithmCollectionBuilder singleton + build() (algorithm_collection_builder.cc:20-50)
  struct B : AlgorithmBuilder {
    Probe* p;
    explicit B(Probe* p) : p(p) {}
    std::shared_ptr<Algorithm> build() override { return probeAlgo("user_ag", "allgather", p); }
  };
  auto inst = collective::AlgorithmCollectionBuilder::getInstance();
  CHECK(inst == collective::AlgorithmCollectionBuilder::getInstance());
  Probe bp;
  inst->addAlgorithmBuilder(std::make_shared<B>(&bp));
  inst->setFallbackAlgorithmSelector(defaultAlgoSelector);
  auto built = inst->build();
  CHECK(built.getAlgorithmsByCollective("allgather").count("user_ag") == 1);
  collective::AlgorithmCollectionBuilder::reset();
  CHECK(collective::AlgorithmCollectionBuilder::getInstance() != inst);
  CHECK(collective::AlgorithmCollectionBuilder::getInstance()->build().getAllAlgorithms().empty());
  CHECK(dataTypeFromNccl(ncclFloat16) == DataType::FLOAT16 && dataTypeFromNccl(ncclBfloat16) == DataType::BFLOAT16 &&
        dataTypeFromNccl(ncclFloat32) == DataType::FLOAT32 && dataTypeFromNccl(ncclInt32) == DataType::INT32 &&
        dataTypeFromNccl(ncclFloat8e4m3) == DataType::FLOAT8_E4M3FN && dataTypeFromNccl(ncclFloat64) == DataType::AUTO);
  std::printf("cpu OK\n");
  return 0;
}

// ---- multi-process GPU part ---------------------------------------------------------------------
// The user allgather: every rank copies its input into every rank's output at offset rank*bytes
// through the peers' mapped outputs, then a host barrier (the reference example's port channels
// do putWithSignal + flush + wait; a copy-engine copy + barrier is the same contract here).
struct AgCtx {
  std::vector<void*> outs;
};
static std::atomic<int> gAgInits{0}, gAgCtxs{0}, gAgCalls{0};

struct UserAllgatherBuilder : AlgorithmBuilder {
  std::shared_ptr<Communicator> comm_;
  std::shared_ptr<Algorithm> build() override {
    return std::make_shared<NativeAlgorithm>(
        "user_allgather", "allgather",
        [this](std::shared_ptr<Communicator> c) {
          comm_ = c;
          gAgInits++;
        },
        [this](const std::shared_ptr<void> ctx, const void* in, void*, size_t inSize, size_t, DataType, ReduceOp,
               hipStream_t s, int, int, const std::unordered_map<std::string, uintptr_t>&, DataType) {
          auto c = std::static_pointer_cast<AgCtx>(ctx);
          gAgCalls++;
          for (size_t r = 0; r < c->outs.size(); ++r)
            if (hipMemcpyAsync((char*)c->outs[r] + (size_t)comm_->rank() * inSize, in, inSize,
                               hipMemcpyDeviceToDevice, s) != hipSuccess)
              return CommResult::CommUnhandledCudaError;
          if (hipStreamSynchronize(s) != hipSuccess) return CommResult::CommUnhandledCudaError;
          comm_->barrier();
          return CommResult::CommSuccess;
        },
        [](std::shared_ptr<Communicator> c, const void*, void* out, size_t, size_t, DataType) {
          gAgCtxs++;
          auto ctx = std::make_shared<AgCtx>();
          ctx->outs = c->registerMemory(out);
          return std::static_pointer_cast<void>(ctx);
        },
        [](const void* in, void* out, size_t is, size_t os, DataType, bool) {
          return AlgorithmCtxKey{const_cast<void*>(in), out, is, os, 0};
        });
  }
};

// e4m3b15 (gpu_data_types.hpp:78-155): sign, 4-bit exponent with bias 15, 3-bit mantissa, no inf/NaN
static double b15Value(int b) {
  const int e = (b >> 3) & 0xf, m = b & 7;
  const double v = e == 0 ? std::ldexp(m / 8.0, -14) : std::ldexp(1.0 + m / 8.0, e - 15);
  return (b & 0x80) ? -v : v;
}
static int b15Exact(double v) {  // the byte that holds v exactly, or -1
  for (int b = 0; b < 256; ++b)
    if (b15Value(b) == v && !(v == 0 && b != 0)) return b;
  return -1;
}
static std::shared_ptr<Algorithm> gBuiltinPacket, gBuiltinRsag;

// uint8 and e4m3b15 through the built-in algorithms' Algorithm::execute, the reference's route for
// DataType::FLOAT8_E4M3B15 (it has no ncclDataType_t): the three accumulation forms, sums exact
static void byteTypesThroughExecute(int rank, int n, hipStream_t s) {
  CHECK(gBuiltinPacket && gBuiltinRsag);
  const size_t bytes = 1 << 16;
  uint8_t *x, *y;
  HIP_OK(hipMalloc(&x, bytes));
  HIP_OK(hipMalloc(&y, bytes));
  std::vector<uint8_t> hx(bytes), hy(bytes);
  for (auto algo : {gBuiltinPacket, gBuiltinRsag}) {
    for (DataType acc : {DataType::AUTO, DataType::FLOAT16, DataType::FLOAT32}) {
      for (size_t i = 0; i < bytes; ++i) hx[i] = (uint8_t)b15Exact(std::ldexp(1.0 + (i % 8) / 8.0, -5 - (int)(i % 5)));
      HIP_OK(hipMemcpy(x, hx.data(), bytes, hipMemcpyHostToDevice));
      CHECK(algo->execute(nullptr, x, y, bytes, bytes, DataType::FLOAT8_E4M3B15, SUM, s, nullptr, 0, 0, false, {},
                          acc) == CommResult::CommSuccess);
      HIP_OK(hipStreamSynchronize(s));
      HIP_OK(hipMemcpy(hy.data(), y, bytes, hipMemcpyDeviceToHost));
      size_t bad = 0;
      for (size_t i = 0; i < bytes; ++i) {
        const int want = b15Exact(n * b15Value(hx[i]));  // n * (1 + m/8) 2^-k: exact for n = 1, 2, 4, 8
        if (want >= 0 && hy[i] != want) bad++;
      }
      if (bad) std::fprintf(stderr, "rank %d %s e4m3b15 accum %d: %zu bad\n", rank, algo->name().c_str(), (int)acc, bad);
      CHECK(bad == 0);
    }
    // uint8: wrapping byte sums (allreduce_test.cu's uint8 check is the same modular sum)
    for (size_t i = 0; i < bytes; ++i) hx[i] = (uint8_t)(rank * 97 + i * 31);
    HIP_OK(hipMemcpy(x, hx.data(), bytes, hipMemcpyHostToDevice));
    CHECK(algo->execute(nullptr, x, y, bytes, bytes, DataType::UINT8, SUM, s, nullptr) == CommResult::CommSuccess);
    HIP_OK(hipStreamSynchronize(s));
    HIP_OK(hipMemcpy(hy.data(), y, bytes, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 0; i < bytes; ++i) {
      unsigned want = 0;
      for (int r = 0; r < n; ++r) want += (uint8_t)(r * 97 + i * 31);
      if (hy[i] != (uint8_t)want) bad++;
    }
    CHECK(bad == 0);
  }
  HIP_OK(hipFree(x));
  HIP_OK(hipFree(y));
}

static int worker(int rank, int n, ncclUniqueId id) {
  int ndev = 0;
  HIP_OK(hipGetDeviceCount(&ndev));
  HIP_OK(hipSetDevice(rank % ndev));
  auto builder = collective::AlgorithmCollectionBuilder::getInstance();
  builder->addAlgorithmBuilder(std::make_shared<UserAllgatherBuilder>());
  // the user selector: allgather -> the user algorithm; allreduce of exactly 3 MiB -> the built-in
  // ring-order RS+AG by name; everything else -> nullptr (the built-in fallback selector)
  builder->setAlgorithmSelector([](const AlgoMapByCollective& m, const CollectiveRequest& r) -> std::shared_ptr<Algorithm> {
    if (r.collective == "allreduce" && !gBuiltinPacket) {
      gBuiltinPacket = m.at("allreduce").at("default_allreduce_packet");
      gBuiltinRsag = m.at("allreduce").at("default_allreduce_rsag");
    }
    if (r.collective == "allgather") return m.at("allgather").at("user_allgather");
    if (r.collective == "allreduce" && r.messageSize == (3u << 20)) return m.at("allreduce").at("default_allreduce_rsag");
    return nullptr;
  });
  ncclComm_t comm;
  NCCL_OK(ncclCommInitRank(&comm, n, id, rank));
  hipStream_t s;
  HIP_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));

  // allgather through the user algorithm, twice on the same buffers (one context)
  const size_t cnt = 1 << 16;
  int *in, *out;
  HIP_OK(hipMalloc(&in, cnt * 4));
  HIP_OK(hipMalloc(&out, cnt * 4 * n));
  std::vector<int> h(cnt), ho(cnt * n);
  for (size_t i = 0; i < cnt; ++i) h[i] = rank * 1000003 + (int)i;
  HIP_OK(hipMemcpy(in, h.data(), cnt * 4, hipMemcpyHostToDevice));
  for (int it = 0; it < 2; ++it) NCCL_OK(ncclAllGather(in, out, cnt, ncclInt32, comm, s));
  HIP_OK(hipStreamSynchronize(s));
  HIP_OK(hipMemcpy(ho.data(), out, ho.size() * 4, hipMemcpyDeviceToHost));
  for (int r = 0; r < n; ++r)
    for (size_t i = 0; i < cnt; ++i) CHECK(ho[(size_t)r * cnt + i] == r * 1000003 + (int)i);
  CHECK(gAgInits == 1 && gAgCtxs == 1 && gAgCalls == 2);

  // allreduce: 3 MiB -> user-selected default_allreduce_rsag; 64 KiB and 4 MiB -> fallback
  // (packet / fullmesh).  int32 input = rank -> n(n-1)/2 (allreduce_test.cu:1172-1183)
  for (size_t bytes : {(size_t)3 << 20, (size_t)64 << 10, (size_t)4 << 20}) {
    const size_t c = bytes / 4;
    int *x, *y;
    HIP_OK(hipMalloc(&x, bytes));
    HIP_OK(hipMalloc(&y, bytes));
    std::vector<int> hx(c, rank), hy(c, -1);
    HIP_OK(hipMemcpy(x, hx.data(), bytes, hipMemcpyHostToDevice));
    NCCL_OK(ncclAllReduce(x, y, c, ncclInt32, ncclSum, comm, s));
    HIP_OK(hipStreamSynchronize(s));
    HIP_OK(hipMemcpy(hy.data(), y, bytes, hipMemcpyDeviceToHost));
    size_t bad = 0, first = c;
    for (size_t i = 0; i < c; ++i)
      if (hy[i] != n * (n - 1) / 2 && bad++ == 0) first = i;
    if (bad)
      std::fprintf(stderr, "rank %d allreduce %zu bytes: %zu bad, first at %zu = %d\n", rank, bytes, bad, first,
                   hy[first]);
    CHECK(bad == 0);
    HIP_OK(hipFree(x));
    HIP_OK(hipFree(y));
  }
  byteTypesThroughExecute(rank, n, s);
  // an unsupported op comes back as an argument error, not a crash
  CHECK(ncclAllReduce(in, in, cnt, ncclInt32, ncclProd, comm, s) == ncclInvalidArgument);
  ncclResult_t async = ncclSuccess;
  NCCL_OK(ncclCommGetAsyncError(comm, &async));
  CHECK(async == ncclSuccess);
  NCCL_OK(ncclCommDestroy(comm));
  HIP_OK(hipFree(in));
  HIP_OK(hipFree(out));
  std::printf("rank %d OK\n", rank);
  std::fflush(stdout);
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 2 && std::string(argv[1]) == "cpu") return runCpu();
  if (argc >= 3 && std::string(argv[1]) == "gpu") {
    const int n = std::atoi(argv[2]);
    ncclUniqueId id;
    NCCL_OK(ncclGetUniqueId(&id));  // the root listens in this (parent) process; no GPU touched here
    std::vector<pid_t> pids;
    for (int r = 0; r < n; ++r) {
      pid_t pid = fork();
      CHECK(pid >= 0);
      if (pid == 0) std::_Exit(worker(r, n, id));
      pids.push_back(pid);
    }
    int bad = 0;
    for (pid_t pid : pids) {
      int st = 0;
      waitpid(pid, &st, 0);
      if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) bad++;
    }
    std::printf(bad ? "gpu FAILED\n" : "gpu OK\n");
    return bad ? 1 : 0;
  }
  std::fprintf(stderr, "usage: %s cpu | gpu <nranks>\n", argv[0]);
  return 2;
}
