// Host core API (include/mscclpp_amd/core.hpp): bootstrap wrapper, registered memory, connections,
// semaphores and the Communicator's connect / send / recv / buildSemaphore, plus the process-wide IPC
// mapping cache every owner of a peer mapping goes through.
//
// Reference behaviour restated (not translated):
//   RegisteredMemory serialize / deserialize   src/core/registered_memory.cc:35-145 (CudaIpc part)
//   IPC open cache                             src/core/gpu_ipc_mem.cc:193-223
//   CudaIpcConnection write / updateAndSync /
//   flush                                      src/core/connection.cc:85-195, context.cc:16-46
//   Communicator connect / sendMemory /
//   recvMemory / buildSemaphore                src/core/communicator.cc:86-173
//   SemaphoreStub / Semaphore                  src/core/semaphore.cc:32-116
#include <unistd.h>

#include <chrono>
#include <condition_variable>
#include <deque>
#include <thread>
#include <random>
#include <unordered_map>

#include "comm_internal.hpp"
#include "mscclpp_amd/core.hpp"
#include "mscclpp_amd/gpu_utils.hpp"
#include "mscclpp_amd/memory_channel.hpp"
#include "mscclpp_amd/semaphore.hpp"

namespace mscclpp_amd {
namespace host {

namespace {
struct HandleKey {
  hipIpcMemHandle_t h;
  bool operator==(const HandleKey& o) const { return std::memcmp(&h, &o.h, sizeof(h)) == 0; }
};
struct HandleKeyHash {
  size_t operator()(const HandleKey& k) const {
    const unsigned char* p = reinterpret_cast<const unsigned char*>(&k.h);
    size_t x = 1469598103934665603ull;
    for (size_t i = 0; i < sizeof(k.h); ++i) x = (x ^ p[i]) * 1099511628211ull;
    return x;
  }
};
std::mutex gIpcMu;
std::unordered_map<HandleKey, std::weak_ptr<void>, HandleKeyHash> gIpcOpen;
// Handles whose mapping is being closed (the closer thread sits in hipIpcCloseMemHandle, which waits
// for the device to go idle).  An open of the same handle meanwhile waits for that close to finish,
// so the handle is never opened while its previous mapping is half torn down.
std::unordered_map<HandleKey, int, HandleKeyHash> gIpcClosing;
std::condition_variable gIpcClosed;
}  // namespace

std::shared_ptr<void> openIpcHandle(const hipIpcMemHandle_t& handle) {
  std::unique_lock<std::mutex> lk(gIpcMu);
  HandleKey key{handle};
  bool warned = false;
  for (;;) {
    // An entry whose mapping has expired belongs to a deleter that has not reached its lock yet:
    // that is a close in progress too.  Only the deleter erases the entry.
    auto it = gIpcOpen.find(key);
    if (it != gIpcOpen.end()) {
      if (auto p = it->second.lock()) return p;  // still mapped (possibly queued for closing: revived)
    } else if (gIpcClosing.find(key) == gIpcClosing.end()) {
      break;
    }
    // rare: a buffer re-registered while its previous mapping is being closed (the close waits for
    // the device to go idle, so a kernel that never ends keeps this waiting: say so once)
    if (gIpcClosed.wait_for(lk, std::chrono::seconds(10)) == std::cv_status::timeout && !warned) {
      warn("openIpcHandle: waiting for the previous mapping of this handle to close (the device is not idle)");
      warned = true;
    }
  }
  void* mapped = nullptr;
  HIPCHECK(hipIpcOpenMemHandle(&mapped, handle, hipIpcMemLazyEnablePeerAccess));
  std::shared_ptr<void> p(mapped, [key](void* q) {
    {
      std::lock_guard<std::mutex> lk2(gIpcMu);
      auto j = gIpcOpen.find(key);
      if (j != gIpcOpen.end() && j->second.expired()) gIpcOpen.erase(j);
      ++gIpcClosing[key];
    }
    const hipError_t e = hipIpcCloseMemHandle(q);
    if (e != hipSuccess) warn(std::string("hipIpcCloseMemHandle: ") + hipGetErrorString(e));
    {
      std::lock_guard<std::mutex> lk2(gIpcMu);
      auto j = gIpcClosing.find(key);
      if (j != gIpcClosing.end() && --j->second <= 0) gIpcClosing.erase(j);
    }
    gIpcClosed.notify_all();
  });
  gIpcOpen[key] = p;
  return p;
}

namespace {
// Mappings whose last user has gone, closed on a thread of their own: hipIpcCloseMemHandle waits for
// the whole device to go idle, so a close on a caller's thread would stall that caller behind every
// stream of the device.  The thread is started on first use and never joined
// (its state is never destroyed, like the pool's): closes still queued at exit are left to the OS.
struct Closer {
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::pair<int, std::shared_ptr<void>>> q;
  size_t inFlight = 0;  // queued or being closed
  bool started = false;
};
Closer& closer() {
  static Closer* c = new Closer();
  return *c;
}
void closerLoop() {
  Closer& c = closer();
  for (;;) {
    std::pair<int, std::shared_ptr<void>> item;
    {
      std::unique_lock<std::mutex> lk(c.mu);
      c.cv.wait(lk, [&] { return !c.q.empty(); });
      item = std::move(c.q.front());
      c.q.pop_front();
    }
    if (item.first >= 0) (void)hipSetDevice(item.first);
    item.second.reset();  // the last reference: the deleter closes the mapping here
    std::lock_guard<std::mutex> lk(c.mu);
    --c.inFlight;
    c.cv.notify_all();
  }
}
// At exit, before the HIP runtime's own teardown (this handler is registered after HIP started):
// let the queued closes finish, for at most 10 s, so no close is still inside HIP when it unloads.
void drainCloser() {
  Closer& c = closer();
  std::unique_lock<std::mutex> lk(c.mu);
  c.cv.wait_for(lk, std::chrono::seconds(10), [&] { return c.inFlight == 0; });
}
}  // namespace

void releaseMappingLater(int device, std::shared_ptr<void> map) {
  if (!map) return;
  Closer& c = closer();
  std::lock_guard<std::mutex> lk(c.mu);
  if (!c.started) {
    std::thread(closerLoop).detach();
    std::atexit(drainCloser);
    c.started = true;
  }
  c.q.emplace_back(device, std::move(map));
  ++c.inFlight;
  c.cv.notify_all();
}

size_t pendingMappingReleases() {
  Closer& c = closer();
  std::lock_guard<std::mutex> lk(c.mu);
  return c.inFlight;
}

size_t liveIpcMappings() {
  std::lock_guard<std::mutex> lk(gIpcMu);
  size_t n = 0;
  for (auto& kv : gIpcOpen) n += kv.second.expired() ? 0 : 1;
  return n;
}

uint64_t processNonce() {
  static const uint64_t nonce = [] {
    std::random_device rd;
    uint64_t v = ((uint64_t)rd() << 32) ^ rd();
    v ^= (uint64_t)getpid() * 0x9e3779b97f4a7c15ull;
    v ^= (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count();
    return v ? v : 1;
  }();
  return nonce;
}

namespace {
// Imports of peers' pooled uncached blocks, kept mapped for the life of this process: the import-side
// twin of the pool (uncached_pool.cpp).  The owner never returns such a block to HIP
// while it runs, so (owner process, base, bytes) names the same memory for as long as the owner
// lives, and a later export of the same block -- a re-created communicator getting the same scratch
// back from the owner's pool -- finds its mapping here instead of opening a new one.  A mapping of
// uncached memory is therefore never closed, so its virtual range is never handed to another
// allocation of this process.  Bounded by the peers' pools (what their blocks peaked at).
struct Kept {
  std::shared_ptr<void> map;
  uint64_t bytes;
};
std::mutex gKeptMu;
std::map<std::pair<uint64_t, uint64_t>, Kept> gKept;  // (owner, base) -> mapping
}  // namespace

std::shared_ptr<void> openIpcImport(const hipIpcMemHandle_t& handle, uint64_t owner, uint64_t base, uint64_t bytes,
                                    bool pooled) {
  static const bool keep = [] {  // diagnosis (tools/portchannel_ab.py): "0" opens every import afresh
    const char* e = std::getenv("MSCCLPP_AMD_IPC_KEEP");
    return !(e && std::string(e) == "0");
  }();
  if (!pooled || !owner || !keep) return openIpcHandle(handle);
  std::lock_guard<std::mutex> lk(gKeptMu);
  const auto key = std::make_pair(owner, base);
  auto it = gKept.find(key);
  if (it != gKept.end()) return it->second.map;
  auto p = openIpcHandle(handle);
  if (!bytes) {  // the caller knows only the registered range: ask HIP for the mapping's extent
    void* b = nullptr;
    size_t sz = 0;
    if (hipMemGetAddressRange((hipDeviceptr_t*)&b, &sz, (hipDeviceptr_t)p.get()) == hipSuccess) bytes = sz;
    else (void)hipGetLastError();
  }
  gKept.emplace(key, Kept{p, bytes});  // never erased: the mapping stays open until the process exits
  return p;
}

size_t releaseKeptIpcImports() {
  std::map<std::pair<uint64_t, uint64_t>, Kept> drop;
  {
    std::lock_guard<std::mutex> lk(gKeptMu);
    drop.swap(gKept);
  }
  return drop.size();  // each mapping closes here unless a live owner (a communicator) still holds it
}

void keptIpcImports(std::vector<std::pair<uint64_t, uint64_t>>* ranges) {
  std::lock_guard<std::mutex> lk(gKeptMu);
  ranges->clear();
  for (const auto& kv : gKept) ranges->emplace_back((uint64_t)kv.second.map.get(), kv.second.bytes);
}

uint64_t allocationId(const void* ptr) {
  unsigned long long id = 0;
  if (hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)ptr) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return (uint64_t)id;
}

}  // namespace host

static RegisteredMemory registerLocal(void* ptr, size_t size, TransportFlags transports, int rank);

// ---- Bootstrap ------------------------------------------------------------------------------------
void Bootstrap::send(const std::vector<char>& data, int peer, int tag) {
  uint64_t n = data.size();
  send(&n, sizeof(n), peer, tag);
  if (n) send(const_cast<char*>(data.data()), (int)n, peer, tag);
}

void Bootstrap::recv(std::vector<char>& data, int peer, int tag) {
  uint64_t n = 0;
  recv(&n, sizeof(n), peer, tag);
  data.resize(n);
  if (n) recv(data.data(), (int)n, peer, tag);
}

namespace {
// The communicator's TCP bootstrap behind the Bootstrap interface (core.hpp:29-110).
class CommBootstrap : public Bootstrap {
 public:
  explicit CommBootstrap(ncclComm_t c) : c_(c) {}
  int getRank() const override { return c_->rank; }
  int getNranks() const override { return c_->nranks; }
  int getNranksPerNode() const override { return c_->nranks; }
  void send(void* data, int size, int peer, int tag) override { c_->boot->send(data, (size_t)size, peer, tag); }
  void recv(void* data, int size, int peer, int tag) override { c_->boot->recv(data, (size_t)size, peer, tag); }
  void allGather(void* allData, int size) override {
    std::vector<char> mine((char*)allData + (size_t)c_->rank * size, (char*)allData + (size_t)(c_->rank + 1) * size);
    c_->boot->allGather(mine.data(), allData, (size_t)size);
  }
  void barrier() override { c_->boot->barrier(); }
  using Bootstrap::recv;
  using Bootstrap::send;

 private:
  ncclComm_t c_;
};

// Bootstrap tag spaces of the exchanges below, so that a user's memory tag 0 and connection tag 0
// never match each other's messages.
int memTag(int tag) { return tag * 4 + 0; }
int connTag(int tag) { return tag * 4 + 1; }
int semTag(int tag) { return tag * 4 + 2; }

constexpr uint32_t kMemMagic = 0x4d524d41;  // "AMRM"
}  // namespace

// ---- RegisteredMemory -------------------------------------------------------------------------------
struct RegisteredMemory::Impl {
  void* data = nullptr;      // usable here
  uint64_t original = 0;     // owner's pointer
  uint64_t size = 0;
  TransportFlags transports;
  int rank = -1;
  int32_t pid = 0;
  hipIpcMemHandle_t handle{};
  uint64_t offset = 0;       // original - allocation base
  uint64_t owner = 0;        // the owner process's processNonce()
  bool pooled = false;       // the allocation is a block of the owner's uncached pool
  bool coherent = false;     // pooled, or host memory (RegisteredMemory::coherent)
  std::shared_ptr<void> map;  // the IPC mapping (received from another process)
};

namespace {
struct MemWire {
  uint32_t magic;
  int32_t rank;
  int32_t pid;
  uint32_t transports;
  uint64_t original;
  uint64_t size;
  uint64_t offset;
  uint64_t owner;
  uint32_t flags;  // bit 0: pooled, bit 1: coherent
  uint32_t pad;
  hipIpcMemHandle_t handle;
};
}  // namespace

void* RegisteredMemory::data() const { return pimpl_ ? pimpl_->data : nullptr; }
void* RegisteredMemory::originalDataPtr() const { return pimpl_ ? (void*)pimpl_->original : nullptr; }
size_t RegisteredMemory::size() const { return pimpl_ ? (size_t)pimpl_->size : 0; }
TransportFlags RegisteredMemory::transports() const { return pimpl_ ? pimpl_->transports : TransportFlags(); }
int RegisteredMemory::rank() const { return pimpl_ ? pimpl_->rank : -1; }
bool RegisteredMemory::coherent() const { return pimpl_ && pimpl_->coherent; }
// Local or remote by the owner's process nonce, not its PID: ranks in separate PID namespaces that
// share the GPU's IPC namespace (containers with host IPC) can share a PID.
bool RegisteredMemory::remote() const { return pimpl_ && pimpl_->owner != host::processNonce(); }

std::vector<char> RegisteredMemory::serialize() const {
  if (!pimpl_) throw Error("serialize: empty RegisteredMemory", ErrorCode::InvalidUsage);
  MemWire w{};
  w.magic = kMemMagic;
  w.rank = pimpl_->rank;
  w.pid = pimpl_->pid;
  w.transports = pimpl_->transports.has(Transport::CudaIpc) ? 1u : 0u;
  w.original = pimpl_->original;
  w.size = pimpl_->size;
  w.offset = pimpl_->offset;
  w.owner = pimpl_->owner;
  w.flags = (pimpl_->pooled ? 1u : 0u) | (pimpl_->coherent ? 2u : 0u);
  w.handle = pimpl_->handle;
  return std::vector<char>((char*)&w, (char*)&w + sizeof(w));
}

RegisteredMemory RegisteredMemory::deserialize(const std::vector<char>& data) {
  MemWire w{};
  if (data.size() != sizeof(w)) throw Error("deserialize: not a RegisteredMemory", ErrorCode::InvalidUsage);
  std::memcpy(&w, data.data(), sizeof(w));
  if (w.magic != kMemMagic) throw Error("deserialize: not a RegisteredMemory", ErrorCode::InvalidUsage);
  auto impl = std::make_shared<Impl>();
  impl->original = w.original;
  impl->size = w.size;
  impl->transports = w.transports ? TransportFlags(Transport::CudaIpc) : TransportFlags();
  impl->rank = w.rank;
  impl->pid = w.pid;
  impl->handle = w.handle;
  impl->offset = w.offset;
  impl->owner = w.owner;
  impl->pooled = (w.flags & 1u) != 0;
  impl->coherent = (w.flags & 2u) != 0;
  if (w.owner == host::processNonce()) {
    impl->data = (void*)w.original;  // same process (in-process ranks): the pointer is usable as is
  } else {
    try {
      impl->map = host::openIpcImport(w.handle, w.owner, w.original - w.offset, 0, impl->pooled);
    } catch (const host::HipError& e) {
      throw Error(std::string("RegisteredMemory::deserialize: ") + e.what(), ErrorCode::SystemError);
    }
    impl->data = (char*)impl->map.get() + w.offset;
  }
  return RegisteredMemory(impl);
}

// ---- Connection --------------------------------------------------------------------------------------
// Creating the connections' copy stream: MSCCLPP_AMD_COPY_STREAM_PRIORITY=high creates it at the device's
// greatest stream priority (an A/B of DESIGN.md §9: whether the hardware scheduler then picks the
// proxy's copies up sooner while other processes' kernels hold the GPU); default: normal priority.
static hipError_t createCopyStream(hipStream_t* s) {
  static const bool high = [] {
    const char* e = std::getenv("MSCCLPP_AMD_COPY_STREAM_PRIORITY");
    return e && std::string(e) == "high";
  }();
  if (!high) return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
  int least = 0, greatest = 0;
  const hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
  if (e != hipSuccess) return e;
  return hipStreamCreateWithPriority(s, hipStreamNonBlocking, greatest);
}

// CudaIpcConnection (connection.cc:85-195): copies on a non-blocking stream of this GPU.  Token
// values of updateAndSync are staged in a pinned ring, one slot per value (HIP reads a pinned source
// when the copy runs, not when it is queued, so one shared word could publish a later value early);
// a slot is reused only after a stream synchronize retired the copies of the previous lap.
// The copy stream of a communicator's connections.  One stream for all of them (the reference's CUDA
// branch, connection.cc:126-130), not one per connection (its HIP branch): HIP multiplexes a
// process's streams onto GPU_MAX_HW_QUEUES (4) hardware queues, and a connection stream that lands
// on the queue of a kernel spinning for that connection's data never runs -- the PortChannel
// all-to-all hung with 4 ranks on one GPU.
struct SharedCopyStream {
  hipStream_t stream = nullptr;
  ~SharedCopyStream() {
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)hipStreamDestroy(stream);
    }
  }
};

struct Connection::Impl {
  int remoteRank = -1;
  int tag = 0;
  int device = 0;
  Device localDevice{DeviceType::GPU, 0};
  int maxWriteQueueSize = -1;
  std::shared_ptr<Context> context;
  std::shared_ptr<SharedCopyStream> copy;
  hipStream_t stream = nullptr;  // copy->stream
  uint64_t* slots = nullptr;
  uint64_t nvals = 0;
  static constexpr uint64_t kSlots = 1024;
  ~Impl() {
    if (stream) (void)hipStreamSynchronize(stream);
    if (slots) (void)hipHostFree(slots);
  }
  void drain(int64_t timeoutUsec) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      const hipError_t e = hipStreamQuery(stream);
      if (e == hipSuccess) return;
      if (e != hipErrorNotReady)
        throw Error(std::string("Connection::flush: ") + hipGetErrorString(e), ErrorCode::SystemError);
      if (timeoutUsec >= 0 &&
          std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count() >
              timeoutUsec)
        throw Error("Connection::flush timed out", ErrorCode::Timeout);
    }
  }
};

void Connection::write(RegisteredMemory dst, uint64_t dstOffset, RegisteredMemory src, uint64_t srcOffset,
                       uint64_t size) {
  if (!pimpl_) throw Error("write on an empty Connection", ErrorCode::InvalidUsage);
  if (dstOffset + size > dst.size() || srcOffset + size > src.size())
    throw Error("Connection::write out of the registered range", ErrorCode::InvalidUsage);
  if (size == 0) return;
  const hipError_t e = hipMemcpyAsync((char*)dst.data() + dstOffset, (char*)src.data() + srcOffset, size,
                                      hipMemcpyDeviceToDevice, pimpl_->stream);
  if (e != hipSuccess) throw Error(std::string("Connection::write: ") + hipGetErrorString(e), ErrorCode::SystemError);
}

// How a token update reaches the peer (MSCCLPP_AMD_TOKEN_WRITE): "memcpy" (default) = an 8-byte
// hipMemcpyAsync H2D from a pinned slot, as the reference (connection.cc:159-177); "writevalue" =
// hipStreamWriteValue64, a stream-ordered write the command processor performs itself (no copy
// engine or blit kernel behind it).  A/B of the two: DESIGN.md §9.
static int tokenWriteMode() {
  static const int m = [] {
    const char* e = std::getenv("MSCCLPP_AMD_TOKEN_WRITE");
    return e && std::string(e) == "writevalue" ? 1 : 0;
  }();
  return m;
}

void Connection::updateAndSync(RegisteredMemory dst, uint64_t dstOffset, uint64_t* src, uint64_t newValue) {
  if (!pimpl_) throw Error("updateAndSync on an empty Connection", ErrorCode::InvalidUsage);
  if (dstOffset + sizeof(uint64_t) > dst.size())
    throw Error("Connection::updateAndSync out of the registered range", ErrorCode::InvalidUsage);
  if (src) *src = newValue;
  Impl& c = *pimpl_;
  if (tokenWriteMode() == 1) {
    const hipError_t e = hipStreamWriteValue64(c.stream, (char*)dst.data() + dstOffset, newValue, 0);
    if (e != hipSuccess)
      throw Error(std::string("Connection::updateAndSync (hipStreamWriteValue64): ") + hipGetErrorString(e),
                  ErrorCode::SystemError);
    return;
  }
  ++c.nvals;
  if (c.nvals % Impl::kSlots == 0) c.drain(-1);
  uint64_t* slot = &c.slots[c.nvals % Impl::kSlots];
  *slot = newValue;
  const hipError_t e =
      hipMemcpyAsync((char*)dst.data() + dstOffset, slot, sizeof(uint64_t), hipMemcpyHostToDevice, c.stream);
  if (e != hipSuccess)
    throw Error(std::string("Connection::updateAndSync: ") + hipGetErrorString(e), ErrorCode::SystemError);
}

void Connection::flush(int64_t timeoutUsec) {
  if (!pimpl_) throw Error("flush on an empty Connection", ErrorCode::InvalidUsage);
  pimpl_->drain(timeoutUsec);
}

Transport Connection::transport() const { return Transport::CudaIpc; }
Transport Connection::remoteTransport() const { return Transport::CudaIpc; }
int Connection::remoteRank() const { return pimpl_ ? pimpl_->remoteRank : -1; }
int Connection::tag() const { return pimpl_ ? pimpl_->tag : -1; }
hipStream_t Connection::stream() const { return pimpl_ ? pimpl_->stream : nullptr; }
std::shared_ptr<Context> Connection::context() const { return pimpl_ ? pimpl_->context : nullptr; }
const Device& Connection::localDevice() const {
  static const Device none{DeviceType::Unknown, -1};
  return pimpl_ ? pimpl_->localDevice : none;
}
int Connection::getMaxWriteQueueSize() const { return pimpl_ ? pimpl_->maxWriteQueueSize : -1; }

// ---- Semaphore ---------------------------------------------------------------------------------------
struct Semaphore::Impl {
  Connection connection;
  RegisteredMemory local;   // my token (the peer signals into it)
  RegisteredMemory remote;  // the peer's token as mapped here
  std::shared_ptr<void> tokenAlloc;  // keeps my token's allocation alive
  uint64_t budget = 0;
  uint32_t* err = nullptr;
};

Connection& Semaphore::connection() { return pimpl_->connection; }
const Connection& Semaphore::connection() const { return pimpl_->connection; }
const RegisteredMemory& Semaphore::localMemory() const { return pimpl_->local; }
const RegisteredMemory& Semaphore::remoteMemory() const { return pimpl_->remote; }

// ---- Communicator ---------------------------------------------------------------------------------------
Communicator::Communicator(ncclComm_t comm) : comm_(comm) {
  if (!comm) throw Error("Communicator: null ncclComm_t", ErrorCode::InvalidUsage);
}

Communicator::~Communicator() {
  if (owned_ && comm_) (void)ncclCommDestroy(comm_);
}

std::shared_ptr<Communicator> Communicator::create(int rank, int nranks, const ncclUniqueId& id) {
  ncclComm_t c = nullptr;
  const ncclResult_t r = ncclCommInitRank(&c, nranks, id, rank);
  if (r != ncclSuccess)
    throw Error(std::string("ncclCommInitRank: ") + ncclGetErrorString(r) + ": " + ncclGetLastError(nullptr),
                ErrorCode::SystemError);
  auto p = std::make_shared<Communicator>(c);
  p->owned_ = true;
  return p;
}

namespace {
std::string initError(ncclResult_t r) {
  return std::string(ncclGetErrorString(r)) + ": " + ncclGetLastError(nullptr);
}
}  // namespace

// ---- TcpBootstrap (core.hpp:113-197) ----------------------------------------------------------------
struct TcpBootstrap::Impl {
  int rank = 0, nranks = 0;
  UniqueId id{};
  bool haveId = false;
  ncclComm_t comm = nullptr;
  std::shared_ptr<Bootstrap> link;  // the communicator's bootstrap (CommBootstrap)
  Bootstrap& ready() const {
    if (!link) throw Error("TcpBootstrap: call initialize() first", ErrorCode::InvalidUsage);
    return *link;
  }
  void init(const void* id128, int64_t timeoutSec) {
    if (comm) throw Error("TcpBootstrap: already initialized", ErrorCode::InvalidUsage);
    const int r = host::commInitRank(&comm, nranks, id128, rank, (int)timeoutSec);
    if (r != ncclSuccess) {
      comm = nullptr;
      throw Error("TcpBootstrap::initialize: " + initError((ncclResult_t)r), ErrorCode::SystemError);
    }
    link = std::make_shared<CommBootstrap>(comm);
  }
};

UniqueId TcpBootstrap::createUniqueId() {
  ncclUniqueId nid;
  const ncclResult_t r = ncclGetUniqueId(&nid);
  if (r != ncclSuccess) throw Error("TcpBootstrap::createUniqueId: " + initError(r), ErrorCode::SystemError);
  UniqueId id;
  static_assert(sizeof(nid) == UniqueIdBytes, "ncclUniqueId and UniqueId are both 128 bytes");
  std::memcpy(id.data(), &nid, UniqueIdBytes);
  return id;
}

TcpBootstrap::TcpBootstrap(int rank, int nRanks) : pimpl_(std::make_unique<Impl>()) {
  if (nRanks <= 0 || rank < 0 || rank >= nRanks)
    throw Error("TcpBootstrap: rank " + std::to_string(rank) + " of " + std::to_string(nRanks), ErrorCode::InvalidUsage);
  pimpl_->rank = rank;
  pimpl_->nranks = nRanks;
}

TcpBootstrap::~TcpBootstrap() {
  if (pimpl_ && pimpl_->comm) (void)ncclCommDestroy(pimpl_->comm);
}

UniqueId TcpBootstrap::getUniqueId() const {
  if (!pimpl_->haveId) throw Error("TcpBootstrap::getUniqueId: no id yet", ErrorCode::InvalidUsage);
  return pimpl_->id;
}

void TcpBootstrap::initialize(UniqueId uniqueId, int64_t timeoutSec) {
  pimpl_->id = uniqueId;
  pimpl_->haveId = true;
  pimpl_->init(uniqueId.data(), timeoutSec);
}

void TcpBootstrap::initialize(const std::string& ifIpPortTrio, int64_t timeoutSec) {
  BootstrapId bid;
  try {
    bid = bootstrapIdFromIpPort(ifIpPortTrio, /*createRoot*/ pimpl_->rank == 0);
  } catch (const std::invalid_argument& e) {
    throw Error(std::string("TcpBootstrap::initialize: ") + e.what(), ErrorCode::InvalidUsage);
  } catch (const std::exception& e) {
    throw Error(std::string("TcpBootstrap::initialize: ") + e.what(), ErrorCode::SystemError);
  }
  std::memcpy(pimpl_->id.data(), &bid, UniqueIdBytes);
  pimpl_->haveId = true;
  pimpl_->init(&bid, timeoutSec);
}

int TcpBootstrap::getRank() const { return pimpl_->rank; }
int TcpBootstrap::getNranks() const { return pimpl_->nranks; }
int TcpBootstrap::getNranksPerNode() const { return pimpl_->nranks; }
void TcpBootstrap::send(void* data, int size, int peer, int tag) { pimpl_->ready().send(data, size, peer, tag); }
void TcpBootstrap::recv(void* data, int size, int peer, int tag) { pimpl_->ready().recv(data, size, peer, tag); }
void TcpBootstrap::allGather(void* allData, int size) { pimpl_->ready().allGather(allData, size); }
void TcpBootstrap::barrier() { pimpl_->ready().barrier(); }
ncclComm_t TcpBootstrap::ncclComm() const { return pimpl_->comm; }

Communicator::Communicator(std::shared_ptr<Bootstrap> bootstrap, std::shared_ptr<Context>) : comm_(nullptr) {
  if (!bootstrap) throw Error("Communicator: null bootstrap", ErrorCode::InvalidUsage);
  if (auto* tcp = dynamic_cast<TcpBootstrap*>(bootstrap.get())) {
    comm_ = tcp->ncclComm();  // owned by the bootstrap, which this communicator keeps alive
    if (!comm_) throw Error("Communicator: the TcpBootstrap is not initialized", ErrorCode::InvalidUsage);
  } else {
    // any other Bootstrap: rank 0's fresh id travels over it, then every rank builds the communicator
    const int rank = bootstrap->getRank(), n = bootstrap->getNranks();
    std::vector<ncclUniqueId> ids((size_t)n);
    if (rank == 0) {
      const ncclResult_t r = ncclGetUniqueId(&ids[0]);
      if (r != ncclSuccess) throw Error("Communicator: ncclGetUniqueId: " + initError(r), ErrorCode::SystemError);
    }
    bootstrap->allGather(ids.data(), (int)sizeof(ncclUniqueId));
    const ncclResult_t r = ncclCommInitRank(&comm_, n, ids[0], rank);
    if (r != ncclSuccess) {
      comm_ = nullptr;
      throw Error("Communicator: ncclCommInitRank: " + initError(r), ErrorCode::SystemError);
    }
    owned_ = true;
  }
  bootstrap_ = std::move(bootstrap);
}

int Communicator::rank() const { return comm_->rank; }
int Communicator::nRanks() const { return comm_->nranks; }
int Communicator::nRanksPerNode() const { return comm_->nranks; }
int Communicator::device() const { return comm_->device; }
uint32_t* Communicator::deviceErrorWord() const { return comm_->err; }
uint64_t Communicator::spinBudget() const { return host::spinBudgetTicks(); }

std::shared_ptr<Bootstrap> Communicator::bootstrap() {
  if (!bootstrap_) bootstrap_ = std::make_shared<CommBootstrap>(comm_);
  return bootstrap_;
}

RegisteredMemory Communicator::registerMemory(void* ptr, size_t size, TransportFlags transports) {
  return registerLocal(ptr, size, transports, comm_->rank);
}

// A registration of this process's buffer; `rank` is the owner's rank (-1: made by a Context).
static RegisteredMemory registerLocal(void* ptr, size_t size, TransportFlags transports, int rank) {
  if (!ptr || size == 0) throw Error("registerMemory: null or empty buffer", ErrorCode::InvalidUsage);
  auto impl = std::make_shared<RegisteredMemory::Impl>();
  impl->data = ptr;
  impl->original = (uint64_t)ptr;
  impl->size = size;
  impl->transports = transports;
  impl->rank = rank;
  impl->pid = (int32_t)getpid();
  impl->owner = host::processNonce();
  {
    hipPointerAttribute_t attr{};
    if (hipPointerGetAttributes(&attr, ptr) == hipSuccess) {
      // host memory (pinned, or pageable: "unregistered" on ROCm 6), and device memory allocated
      // fine-grained or uncached (hipExtMallocWithFlags: both flags carry the fine-grained bit) are
      // coherent with the proxy's copies; the pool's blocks are recognised below
      impl->coherent = attr.type == hipMemoryTypeHost || attr.type == hipMemoryTypeUnregistered ||
                       (attr.type == hipMemoryTypeDevice && (attr.allocationFlags & hipDeviceMallocFinegrained) != 0);
    } else {
      (void)hipGetLastError();
      impl->coherent = true;  // pageable host memory, unknown to HIP
    }
  }
  if (transports.has(Transport::CudaIpc)) {
    void* base = nullptr;
    size_t range = 0;
    hipError_t e = hipMemGetAddressRange((hipDeviceptr_t*)&base, &range, (hipDeviceptr_t)ptr);
    if (e == hipSuccess && (char*)ptr + size > (char*)base + range) e = hipErrorInvalidValue;
    if (e == hipSuccess) e = hipIpcGetMemHandle(&impl->handle, base);
    if (e != hipSuccess)
      throw Error(std::string("registerMemory: not a device allocation (") + hipGetErrorString(e) + ")",
                  ErrorCode::InvalidUsage);
    impl->offset = (uint64_t)((char*)ptr - (char*)base);
    impl->pooled = host::isPooledUncached(base);
    if (impl->pooled) impl->coherent = true;
  }
  return RegisteredMemory(impl);
}

void Communicator::sendMemory(RegisteredMemory memory, int remoteRank, int tag) {
  bootstrap()->send(memory.serialize(), remoteRank, memTag(tag));
}

std::shared_future<RegisteredMemory> Communicator::recvMemory(int remoteRank, int tag) {
  auto boot = bootstrap();
  return std::async(std::launch::deferred, [boot, remoteRank, tag] {
           std::vector<char> data;
           boot->recv(data, remoteRank, memTag(tag));
           return RegisteredMemory::deserialize(data);
         }).share();
}

namespace {
struct EndpointWire {
  int32_t rank;
  int32_t pid;
  int32_t device;
  int32_t transport;
};
}  // namespace

std::shared_future<Connection> Communicator::connect(const EndpointConfig& localConfig, int remoteRank, int tag) {
  if (localConfig.transport != Transport::CudaIpc)
    throw Error("connect: one MI355X node carries CudaIpc connections only", ErrorCode::InvalidUsage);
  if (localConfig.device.type != DeviceType::GPU ||
      (localConfig.device.id >= 0 && localConfig.device.id != comm_->device))
    throw Error("connect: the local endpoint is this communicator's GPU (" + std::to_string(comm_->device) + ")",
                ErrorCode::InvalidUsage);
  if (remoteRank < 0 || remoteRank >= comm_->nranks)
    throw Error("connect: bad remote rank", ErrorCode::InvalidUsage);
  EndpointWire mine{comm_->rank, (int32_t)getpid(), comm_->device, (int32_t)Transport::CudaIpc};
  auto boot = bootstrap();
  boot->send(&mine, (int)sizeof(mine), remoteRank, connTag(tag));
  const int device = comm_->device;
  std::shared_ptr<SharedCopyStream> copy;
  {
    std::lock_guard<std::mutex> lk(comm_->ipcStreamMu);
    copy = std::static_pointer_cast<SharedCopyStream>(comm_->ipcStream.lock());
    if (!copy) {
      copy = std::make_shared<SharedCopyStream>();
      int cur = 0;
      gpuCheck(hipGetDevice(&cur), "hipGetDevice");
      gpuCheck(hipSetDevice(device), "hipSetDevice");
      const hipError_t e = createCopyStream(&copy->stream);
      gpuCheck(hipSetDevice(cur), "hipSetDevice");
      gpuCheck(e, "hipStreamCreateWithFlags");
      comm_->ipcStream = copy;
    }
  }
  auto ctx = context();
  const int maxWq = localConfig.maxWriteQueueSize;
  return std::async(std::launch::deferred, [boot, remoteRank, tag, device, copy, ctx, maxWq] {
           EndpointWire peer{};
           boot->recv(&peer, (int)sizeof(peer), remoteRank, connTag(tag));
           if (peer.transport != (int32_t)Transport::CudaIpc)
             throw Error("connect: the peer offered another transport", ErrorCode::InvalidUsage);
           auto impl = std::make_shared<Connection::Impl>();
           impl->remoteRank = remoteRank;
           impl->tag = tag;
           impl->device = device;
           impl->localDevice = Device(DeviceType::GPU, device);
           impl->maxWriteQueueSize = maxWq;
           impl->context = ctx;
           int cur = 0;
           gpuCheck(hipGetDevice(&cur), "hipGetDevice");
           gpuCheck(hipSetDevice(device), "hipSetDevice");
           impl->copy = copy;
           impl->stream = copy->stream;
           gpuCheck(hipHostMalloc((void**)&impl->slots, Connection::Impl::kSlots * sizeof(uint64_t),
                                  hipHostMallocDefault),
                    "hipHostMalloc");
           gpuCheck(hipSetDevice(cur), "hipSetDevice");
           return Connection(impl);
         }).share();
}

std::shared_future<Connection> Communicator::connect(const Endpoint& localEndpoint, int remoteRank, int tag) {
  if (!localEndpoint.valid()) throw Error("connect: empty endpoint", ErrorCode::InvalidUsage);
  if (localEndpoint.pidHash() != host::processNonce())
    throw Error("connect: the local endpoint belongs to another process", ErrorCode::InvalidUsage);
  return connect(localEndpoint.config(), remoteRank, tag);
}

std::shared_ptr<Context> Communicator::context() {
  if (!context_) context_ = Context::create();
  return context_;
}

int Communicator::remoteRankOf(const Connection& connection) { return connection.remoteRank(); }
int Communicator::tagOf(const Connection& connection) { return connection.tag(); }

std::shared_future<Semaphore> Communicator::buildSemaphore(const Connection& connection, int remoteRank, int tag) {
  if (!connection.valid()) throw Error("buildSemaphore: empty connection", ErrorCode::InvalidUsage);
  // my token: 8 bytes of uncached device memory (semaphore.cc:32-43), registered and sent
  void* tok = host::allocUncached(64);
  std::shared_ptr<void> tokAlloc(tok, [](void* p) { host::freeDevice(p); });
  RegisteredMemory local = registerMemory(tok, sizeof(uint64_t), Transport::CudaIpc);
  auto boot = bootstrap();
  boot->send(local.serialize(), remoteRank, semTag(tag));
  const uint64_t budget = host::spinBudgetTicks();
  uint32_t* err = comm_->err;
  return std::async(std::launch::deferred, [boot, remoteRank, tag, connection, local, tokAlloc, budget, err] {
           std::vector<char> data;
           boot->recv(data, remoteRank, semTag(tag));
           auto impl = std::make_shared<Semaphore::Impl>();
           impl->connection = connection;
           impl->local = local;
           impl->remote = RegisteredMemory::deserialize(data);
           impl->tokenAlloc = tokAlloc;
           impl->budget = budget;
           impl->err = err;
           return Semaphore(impl);
         }).share();
}

std::vector<void*> Communicator::registerMemory(void* ptr) {
  if (!ptr) throw std::invalid_argument("registerMemory: null pointer");
  std::vector<void*> res((size_t)comm_->nranks, nullptr);
  if (comm_->nranks == 1) {
    res[0] = ptr;
    return res;
  }
  std::lock_guard<std::mutex> lk(comm_->mu);
  // collective IPC exchange, cached per allocation; pinned: the caller keeps these pointers
  auto peers = comm_->registerOutput(ptr, nullptr, /*pin=*/true);
  for (int r = 0; r < comm_->nranks; ++r) res[(size_t)r] = peers[(size_t)r];
  return res;
}

void Communicator::allGather(const void* sendbuf, void* recvbuf, size_t bytesPerRank) {
  comm_->boot->allGather(sendbuf, recvbuf, bytesPerRank);
}

void Communicator::barrier() { comm_->boot->barrier(); }

// ---- semaphores (semaphore.hpp; semaphore.cc:118-238) ---------------------------------------------
Host2DeviceSemaphore::Host2DeviceSemaphore(const Semaphore& semaphore, uint64_t budget, uint32_t* err)
    : semaphore_(semaphore) {
  if (!semaphore.valid()) throw Error("Host2DeviceSemaphore: empty Semaphore", ErrorCode::InvalidUsage);
  gpuCheck(hipMalloc((void**)&expectedInboundToken_, sizeof(uint64_t)), "hipMalloc");
  try {
    memsetSync(expectedInboundToken_, 0, sizeof(uint64_t));
  } catch (...) {  // the destructor does not run for a throwing constructor
    (void)hipFree(expectedInboundToken_);
    throw;
  }
  budget_ = budget ? budget : semaphore.pimpl()->budget;
  err_ = err ? err : semaphore.pimpl()->err;
}

Host2DeviceSemaphore::Host2DeviceSemaphore(Communicator& communicator, const Connection& connection)
    : Host2DeviceSemaphore(communicator.buildSemaphore(connection, connection.remoteRank(), connection.tag()).get()) {}

Host2DeviceSemaphore::~Host2DeviceSemaphore() {
  if (expectedInboundToken_) freeDevice(expectedInboundToken_);
}

Connection& Host2DeviceSemaphore::connection() { return semaphore_.connection(); }

void Host2DeviceSemaphore::signal() {
  semaphore_.connection().updateAndSync(semaphore_.remoteMemory(), 0, &outbound_, outbound_ + 1);
}

Host2DeviceSemaphore::DeviceHandle Host2DeviceSemaphore::deviceHandle() const {
  DeviceHandle h{};
  h.inboundToken = (uint64_t*)semaphore_.localMemory().data();
  h.expectedInboundToken = expectedInboundToken_;
  h.budget = budget_;
  h.err = err_;
  return h;
}

MemoryDevice2DeviceSemaphore::MemoryDevice2DeviceSemaphore(const Semaphore& semaphore, uint64_t budget, uint32_t* err)
    : semaphore_(semaphore) {
  if (!semaphore.valid()) throw Error("MemoryDevice2DeviceSemaphore: empty Semaphore", ErrorCode::InvalidUsage);
  gpuCheck(hipMalloc((void**)&expectedInboundToken_, sizeof(uint64_t)), "hipMalloc");
  try {
    memsetSync(expectedInboundToken_, 0, sizeof(uint64_t));
  } catch (...) {  // the destructor does not run for a throwing constructor
    (void)hipFree(expectedInboundToken_);
    throw;
  }
  budget_ = budget ? budget : semaphore.pimpl()->budget;
  err_ = err ? err : semaphore.pimpl()->err;
}

MemoryDevice2DeviceSemaphore::MemoryDevice2DeviceSemaphore(Communicator& communicator, const Connection& connection)
    : MemoryDevice2DeviceSemaphore(
          communicator.buildSemaphore(connection, connection.remoteRank(), connection.tag()).get()) {}

MemoryDevice2DeviceSemaphore::~MemoryDevice2DeviceSemaphore() {
  if (expectedInboundToken_) freeDevice(expectedInboundToken_);
}

Connection& MemoryDevice2DeviceSemaphore::connection() { return semaphore_.connection(); }

MemoryDevice2DeviceSemaphore::DeviceHandle MemoryDevice2DeviceSemaphore::deviceHandle() const {
  DeviceHandle h{};
  h.inboundToken = (uint64_t*)semaphore_.localMemory().data();
  h.remoteInboundToken = (uint64_t*)semaphore_.remoteMemory().data();
  h.expectedInboundToken = expectedInboundToken_;
  h.budget = budget_;
  h.err = err_;
  return h;
}

BaseMemoryChannel::BaseMemoryChannel(const Semaphore& semaphore)
    : semaphore_(std::make_shared<MemoryDevice2DeviceSemaphore>(semaphore)) {}


// ---- Endpoint / Context / SemaphoreStub (core.hpp:473-690) --------------------------------------------
namespace {
constexpr uint32_t kEndpointMagic = 0x50444e45;  // "ENDP"
struct EndpointWireV2 {
  uint32_t magic;
  int32_t transport, devType, devId, maxWriteQueueSize, pad;
  uint64_t hostHash, pidHash;
};
uint64_t thisHostHash() {
  static const uint64_t h = [] {
    char name[256] = {};
    (void)gethostname(name, sizeof(name) - 1);
    uint64_t x = 1469598103934665603ull;
    for (const char* c = name; *c; ++c) x = (x ^ (unsigned char)*c) * 1099511628211ull;
    return x;
  }();
  return h;
}
}  // namespace

struct Endpoint::Impl {
  EndpointConfig config;
  uint64_t hostHash = 0, pidHash = 0;
};

const EndpointConfig& Endpoint::config() const {
  if (!pimpl_) throw Error("Endpoint: empty", ErrorCode::InvalidUsage);
  return pimpl_->config;
}
Transport Endpoint::transport() const { return config().transport; }
const Device& Endpoint::device() const { return config().device; }
uint64_t Endpoint::hostHash() const { return pimpl_ ? pimpl_->hostHash : 0; }
uint64_t Endpoint::pidHash() const { return pimpl_ ? pimpl_->pidHash : 0; }
int Endpoint::maxWriteQueueSize() const { return config().maxWriteQueueSize; }

std::vector<char> Endpoint::serialize() const {
  const EndpointConfig& c = config();
  EndpointWireV2 w{kEndpointMagic, (int32_t)c.transport, (int32_t)c.device.type, c.device.id, c.maxWriteQueueSize, 0,
                   pimpl_->hostHash, pimpl_->pidHash};
  return std::vector<char>((const char*)&w, (const char*)&w + sizeof(w));
}

Endpoint Endpoint::deserialize(const std::vector<char>& data) {
  EndpointWireV2 w{};
  if (data.size() != sizeof(w)) throw Error("Endpoint::deserialize: bad size", ErrorCode::InvalidUsage);
  std::memcpy(&w, data.data(), sizeof(w));
  if (w.magic != kEndpointMagic) throw Error("Endpoint::deserialize: not an endpoint", ErrorCode::InvalidUsage);
  auto impl = std::make_shared<Endpoint::Impl>();
  impl->config = EndpointConfig((Transport)w.transport, Device((DeviceType)w.devType, w.devId), w.maxWriteQueueSize);
  impl->hostHash = w.hostHash;
  impl->pidHash = w.pidHash;
  return Endpoint(impl);
}

struct Context::Impl {
  std::mutex mu;
  std::map<int, std::shared_ptr<SharedCopyStream>> copy;  // per local GPU: the connections' copy stream
};

Context::Context() : pimpl_(std::make_unique<Impl>()) {}
Context::~Context() = default;
std::shared_ptr<Context> Context::create() { return std::shared_ptr<Context>(new Context()); }

RegisteredMemory Context::registerMemory(void* ptr, size_t size, TransportFlags transports) {
  return registerLocal(ptr, size, transports, -1);
}

Endpoint Context::createEndpoint(EndpointConfig config) {
  if (config.transport != Transport::CudaIpc)
    throw Error("createEndpoint: one MI355X node carries CudaIpc connections only", ErrorCode::InvalidUsage);
  if (config.device.type != DeviceType::GPU)
    throw Error("createEndpoint: CudaIpc endpoints are GPUs", ErrorCode::InvalidUsage);
  if (config.device.id < 0) gpuCheck(hipGetDevice(&config.device.id), "hipGetDevice");
  int n = 0;
  gpuCheck(hipGetDeviceCount(&n), "hipGetDeviceCount");
  if (config.device.id >= n) throw Error("createEndpoint: no GPU " + std::to_string(config.device.id), ErrorCode::InvalidUsage);
  auto impl = std::make_shared<Endpoint::Impl>();
  impl->config = config;
  impl->hostHash = thisHostHash();
  impl->pidHash = host::processNonce();
  return Endpoint(impl);
}

Connection Context::connect(const Endpoint& localEndpoint, const Endpoint& remoteEndpoint) {
  if (!localEndpoint.valid() || !remoteEndpoint.valid()) throw Error("connect: empty endpoint", ErrorCode::InvalidUsage);
  if (localEndpoint.pidHash() != host::processNonce())
    throw Error("connect: the local endpoint belongs to another process", ErrorCode::InvalidUsage);
  if (localEndpoint.transport() != Transport::CudaIpc || remoteEndpoint.transport() != Transport::CudaIpc)
    throw Error("connect: CudaIpc endpoints only", ErrorCode::InvalidUsage);
  if (remoteEndpoint.hostHash() != localEndpoint.hostHash())
    throw Error("connect: the remote endpoint is on another host (one node here)", ErrorCode::InvalidUsage);
  const int dev = localEndpoint.device().id;
  int cur = 0;
  gpuCheck(hipGetDevice(&cur), "hipGetDevice");
  gpuCheck(hipSetDevice(dev), "hipSetDevice");
  auto restore = [&] { (void)hipSetDevice(cur); };
  try {
    const int rdev = remoteEndpoint.device().id;
    if (remoteEndpoint.pidHash() == localEndpoint.pidHash() && rdev != dev) {
      // two GPUs of this process: this GPU stores into the other's memory directly
      const hipError_t e = hipDeviceEnablePeerAccess(rdev, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
        throw Error(std::string("connect: peer access GPU ") + std::to_string(dev) + " -> " + std::to_string(rdev) +
                        ": " + hipGetErrorString(e),
                    ErrorCode::SystemError);
      (void)hipGetLastError();
    }
    std::shared_ptr<SharedCopyStream> copy;
    {
      std::lock_guard<std::mutex> lk(pimpl_->mu);
      auto& slot = pimpl_->copy[dev];
      if (!slot) {
        slot = std::make_shared<SharedCopyStream>();
        gpuCheck(createCopyStream(&slot->stream), "hipStreamCreateWithFlags");
      }
      copy = slot;
    }
    auto impl = std::make_shared<Connection::Impl>();
    impl->device = dev;
    impl->localDevice = Device(DeviceType::GPU, dev);
    impl->maxWriteQueueSize = localEndpoint.maxWriteQueueSize();
    impl->context = shared_from_this();
    impl->copy = copy;
    impl->stream = copy->stream;
    gpuCheck(hipHostMalloc((void**)&impl->slots, Connection::Impl::kSlots * sizeof(uint64_t), hipHostMallocDefault),
             "hipHostMalloc");
    restore();
    return Connection(impl);
  } catch (...) {
    restore();
    throw;
  }
}

struct SemaphoreStub::Impl {
  Connection connection;               // empty for a stub received from elsewhere
  RegisteredMemory memory;             // the token
  std::shared_ptr<void> tokenAlloc;    // the token's allocation (local stubs)
};

SemaphoreStub::SemaphoreStub(const Connection& connection) : pimpl_(std::make_shared<Impl>()) {
  if (!connection.valid()) throw Error("SemaphoreStub: empty connection", ErrorCode::InvalidUsage);
  const int dev = connection.localDevice().id;
  int cur = 0;
  gpuCheck(hipGetDevice(&cur), "hipGetDevice");
  gpuCheck(hipSetDevice(dev), "hipSetDevice");
  void* tok = nullptr;
  try {
    tok = host::allocUncached(64);  // semaphore.cc:32-43: the token in uncached memory on AMD
  } catch (...) {
    (void)hipSetDevice(cur);
    throw;
  }
  (void)hipSetDevice(cur);
  pimpl_->tokenAlloc = std::shared_ptr<void>(tok, [](void* p) { host::freeDevice(p); });
  pimpl_->connection = connection;
  pimpl_->memory = registerLocal(tok, sizeof(uint64_t), Transport::CudaIpc, -1);
}

const RegisteredMemory& SemaphoreStub::memory() const { return pimpl_->memory; }
std::vector<char> SemaphoreStub::serialize() const { return pimpl_->memory.serialize(); }
SemaphoreStub SemaphoreStub::deserialize(const std::vector<char>& data) {
  auto impl = std::make_shared<Impl>();
  impl->memory = RegisteredMemory::deserialize(data);
  return SemaphoreStub(impl);
}

Semaphore::Semaphore(const SemaphoreStub& localStub, const SemaphoreStub& remoteStub) {
  const auto& l = localStub.pimpl();
  const auto& r = remoteStub.pimpl();
  if (!l || !r || !l->connection.valid())
    throw Error("Semaphore: the local stub must be made from a connection of this process", ErrorCode::InvalidUsage);
  auto impl = std::make_shared<Semaphore::Impl>();
  impl->connection = l->connection;
  impl->local = l->memory;
  impl->remote = r->memory;
  impl->tokenAlloc = l->tokenAlloc;
  impl->budget = host::spinBudgetTicks();
  impl->err = nullptr;
  pimpl_ = impl;
}

}  // namespace mscclpp_amd
