// Host side of the proxy transport (include/mscclpp_amd/{fifo,proxy,port_channel}.hpp): the
// trigger FIFO, the proxy thread and the general ProxyService behind PortChannels.
//
// Reference behaviour restated:
//   Fifo::poll / pop                  src/core/fifo.cc:58-78 (commit bit = lap parity, cleared on read)
//   Proxy::start loop                 src/core/proxy.cc:42-100 (busy poll, handler, pop; NUMA bind :23-33)
//   ProxyService::handleTrigger       src/core/port_channel.cc:117-154 (Data -> write, Flag -> signal,
//                                     Sync -> flush, then flushDonePos = position + 1, :155-178)
//   ProxyService::buildAndAddSemaphore / addMemory / portChannel   port_channel.cc:32-90
#include <sched.h>

#include <chrono>
#include <fstream>
#include <sstream>

#include "comm_internal.hpp"
#include "mscclpp_amd/device.hpp"
#include "mscclpp_amd/gpu_utils.hpp"
#include "mscclpp_amd/port_channel.hpp"

namespace mscclpp_amd {

// ---- NUMA (numa.cc / proxy.cc:23-33) ----------------------------------------------------------------
int getDeviceNumaNode(int device) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) return -1;
  std::string id(bus);
  for (auto& ch : id) ch = (char)std::tolower(ch);
  std::ifstream f("/sys/bus/pci/devices/" + id + "/numa_node");
  int node = -1;
  if (f) f >> node;
  return node;
}

int numaBind(int node) {
  if (node < 0) return -1;
  std::ifstream f("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist");
  std::string list;
  if (!f || !std::getline(f, list)) return -1;
  cpu_set_t set;
  CPU_ZERO(&set);
  int count = 0;
  std::stringstream ss(list);
  std::string part;
  while (std::getline(ss, part, ',')) {
    int a = 0, b = 0;
    if (sscanf(part.c_str(), "%d-%d", &a, &b) == 2) {
      for (int c = a; c <= b; ++c, ++count) CPU_SET(c, &set);
    } else if (sscanf(part.c_str(), "%d", &a) == 1) {
      CPU_SET(a, &set);
      ++count;
    }
  }
  if (count == 0) return -1;
  return sched_setaffinity(0, sizeof(set), &set) == 0 ? node : -1;
}

// ---- Fifo ---------------------------------------------------------------------------------------------
Fifo::Fifo(int size) : size_(size) {
  if (size <= 0 || (size & (size - 1))) throw Error("FIFO size must be a power of two", ErrorCode::InvalidUsage);
  while ((1 << shift_) < size) ++shift_;
  const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
  gpuCheck(hipHostMalloc((void**)&triggers_, sizeof(ProxyTrigger) * size, fl), "hipHostMalloc");
  std::memset((void*)triggers_, 0, sizeof(ProxyTrigger) * size);
  gpuCheck(hipHostMalloc((void**)&tail_, 64, fl), "hipHostMalloc");
  std::memset((void*)tail_, 0, 64);
  gpuCheck(hipHostGetDevicePointer((void**)&dTriggers_, (void*)triggers_, 0), "hipHostGetDevicePointer");
  gpuCheck(hipHostGetDevicePointer((void**)&dTail_, (void*)tail_, 0), "hipHostGetDevicePointer");
  gpuCheck(hipMalloc((void**)&head_, 64), "hipMalloc");
  memsetSync(head_, 0, 64);
  gpuCheck(hipMalloc((void**)&tailCache_, 64), "hipMalloc");
  memsetSync(tailCache_, 0, 64);
}

Fifo::~Fifo() {
  (void)hipHostFree((void*)triggers_);
  (void)hipHostFree((void*)tail_);
  freeDevice(head_);
  freeDevice(tailCache_);
}

bool Fifo::poll(ProxyTrigger& t) {
  const uint64_t cur = *tail_;
  ProxyTrigger* slot = &triggers_[cur & (uint64_t)(size_ - 1)];
  const uint64_t snd = __atomic_load_n(&slot->snd, __ATOMIC_ACQUIRE);
  const uint64_t parity = ((cur >> shift_) & 1ull) ^ 1ull;
  if ((snd >> 63) != parity) return false;
  t.snd = snd & ~(1ull << 63);
  t.fst = __atomic_load_n(&slot->fst, __ATOMIC_RELAXED);
  return true;
}

void Fifo::pop() { __atomic_store_n(tail_, *tail_ + 1, __ATOMIC_RELEASE); }

uint64_t Fifo::tail() const { return *tail_; }

FifoDeviceHandle Fifo::deviceHandle(uint64_t budget, uint32_t* err) const {
  FifoDeviceHandle h{};
  h.triggers = dTriggers_;
  h.head = head_;
  h.tail = dTail_;
  h.tailCache = tailCache_;
  h.size = size_;
  h.sizeMask = (uint64_t)size_ - 1;
  h.sizeShift = (uint64_t)shift_;
  h.budget = budget;
  h.err = err;
  return h;
}

// ---- Proxy --------------------------------------------------------------------------------------------
Proxy::Proxy(Handler handler, int fifoSize) : fifo_(fifoSize), handler_(std::move(handler)) {
  gpuCheck(hipGetDevice(&device_), "hipGetDevice");
}

Proxy::~Proxy() { stop(); }

void Proxy::start(bool blocking) {
  if (thread_.joinable()) return;
  running_.store(true, std::memory_order_release);
  thread_ = std::thread([this] {
    (void)hipSetDevice(device_);
    numaNode_ = numaBind(getDeviceNumaNode(device_));
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    (void)hipThreadExchangeStreamCaptureMode(&mode);  // never capture in a proxy thread
    started_.store(true, std::memory_order_release);
    ProxyTrigger t;
    int runCnt = 4096;
    static const bool gapStats = [] {
      const char* e = std::getenv("MSCCLPP_AMD_PROXY_GAP_STATS");
      return e && *e == '1';
    }();
    auto last = std::chrono::steady_clock::now();
    for (;;) {
      if (gapStats) {
        const auto now = std::chrono::steady_clock::now();
        const uint64_t gap = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(now - last).count();
        last = now;
        if (resetGap_.exchange(false, std::memory_order_relaxed)) maxGapNs_.store(0, std::memory_order_relaxed);
        else if (gap > maxGapNs_.load(std::memory_order_relaxed)) maxGapNs_.store(gap, std::memory_order_relaxed);
      }
      if (runCnt-- == 0) {
        runCnt = 4096;
        if (!running_.load(std::memory_order_acquire)) break;
      }
      if (!fifo_.poll(t)) continue;
      const ProxyHandlerResult r = handler_(t, fifo_.tail());
      fifo_.pop();
      if (r == ProxyHandlerResult::Stop) break;
    }
  });
  if (blocking)
    while (!started_.load(std::memory_order_acquire)) std::this_thread::sleep_for(std::chrono::microseconds(50));
}

void Proxy::stop() {
  if (thread_.joinable()) {
    running_.store(false, std::memory_order_release);
    thread_.join();
  }
}

// ---- ProxyService -------------------------------------------------------------------------------------
// Per connection: the pinned, device-mapped word the device's waitFlush polls.
struct ProxyService::ConnState {
  uint64_t* flushDone = nullptr;   // host
  uint64_t* dFlushDone = nullptr;  // device view
  ConnState() {
    gpuCheck(hipHostMalloc((void**)&flushDone, 64, hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc");
    std::memset(flushDone, 0, 64);
    gpuCheck(hipHostGetDevicePointer((void**)&dFlushDone, flushDone, 0), "hipHostGetDevicePointer");
  }
  ~ConnState() { (void)hipHostFree(flushDone); }
};

ProxyService::ProxyService(int fifoSize) {
  proxy_ = std::make_shared<Proxy>([this](ProxyTrigger t, uint64_t pos) { return handleTrigger(t, pos); }, fifoSize);
}

ProxyService::~ProxyService() {
  stopProxy();
  for (void* e : stampEvents_) (void)hipEventDestroy((hipEvent_t)e);
}

void ProxyService::enableStamps(size_t cap) {
  if (cap > (1u << 20)) throw Error("ProxyService::enableStamps: at most 2^20 stamps", ErrorCode::InvalidUsage);
  stamps_.clear();
  stamps_.reserve(cap);
  while (stampEvents_.size() < 2 * cap) {
    hipEvent_t e = nullptr;
    gpuCheck(hipEventCreate(&e), "hipEventCreate");
    stampEvents_.push_back((void*)e);
  }
  stampCap_ = cap;
}

SemaphoreId ProxyService::buildAndAddSemaphore(Communicator& communicator, const Connection& connection) {
  if (!err_) err_ = communicator.deviceErrorWord();
  budget_ = communicator.spinBudget();
  return addSemaphore(std::make_shared<Host2DeviceSemaphore>(communicator, connection));
}

SemaphoreId ProxyService::addSemaphore(const Semaphore& semaphore) {
  return addSemaphore(std::make_shared<Host2DeviceSemaphore>(semaphore));
}

SemaphoreId ProxyService::addSemaphore(std::shared_ptr<Host2DeviceSemaphore> semaphore) {
  if (semaphores_.size() >= (1u << TriggerBitsSemaphoreId))
    throw Error("ProxyService: too many semaphores for the trigger's 10-bit id", ErrorCode::InvalidUsage);
  if (!err_) err_ = semaphore->deviceHandle().err;
  const void* key = semaphore->connection().impl().get();
  auto it = conns_.find(key);
  if (it == conns_.end()) it = conns_.emplace(key, std::make_shared<ConnState>()).first;
  semaphores_.push_back(std::move(semaphore));
  semConn_.push_back(it->second);
  return (SemaphoreId)(semaphores_.size() - 1);
}

static int portChannelDstPolicy();

MemoryId ProxyService::addMemory(RegisteredMemory memory) {
  if (memories_.size() >= (1u << TriggerBitsMemoryId))
    throw Error("ProxyService: too many memories for the trigger's 9-bit id", ErrorCode::InvalidUsage);
  // strict: a peer's cached buffer is refused as soon as it is added -- before any semaphore is built
  // with that peer, so every rank refuses before it could wait in the bootstrap for another
  if (memory.remote() && !memory.coherent() && portChannelDstPolicy() == 2)
    throw Error("ProxyService::addMemory: rank " + std::to_string(memory.rank()) +
                    "'s buffer is cached device memory, refused as a PortChannel destination "
                    "(MSCCLPP_AMD_PORT_CHANNEL_DST=strict; allocate it with GpuBuffer / mscclppAmdMallocUncached)",
                ErrorCode::InvalidUsage);
  memories_.push_back(std::move(memory));
  return (MemoryId)(memories_.size() - 1);
}

MemoryId ProxyService::nextMemoryId(uint32_t count) const {
  if (memories_.size() + count > (1u << TriggerBitsMemoryId))
    throw Error("ProxyService: out of memory ids", ErrorCode::InvalidUsage);
  return (MemoryId)memories_.size();
}

std::shared_ptr<Host2DeviceSemaphore> ProxyService::semaphore(SemaphoreId id) const { return semaphores_.at(id); }

BasePortChannel ProxyService::basePortChannel(SemaphoreId id) {
  return BasePortChannel(id, semaphores_.at(id), proxy_, semConn_.at(id)->dFlushDone);
}

// The destination contract of a PortChannel.  The proxy's copy
// engine writes the destination behind the receiving GPU's L2, so a kernel that is running when the
// data lands reads it reliably only from coherent memory: the uncached pool (GpuBuffer,
// mscclppAmdMallocUncached -- what the reference's PortChannel tests allocate on AMD,
// port_channel_tests.cu:209, :241) or host memory.  Data put into cached device memory (hipMalloc,
// torch) is complete for the host and for kernels launched after the receiving one, as the
// reference's customized AllGather example uses it.  MSCCLPP_AMD_PORT_CHANNEL_DST chooses what a
// non-coherent destination gets: "warn" (default: one warning per ProxyService), "strict"
// (InvalidUsage) or "off".
static int portChannelDstPolicy() {
  const char* e = std::getenv("MSCCLPP_AMD_PORT_CHANNEL_DST");
  if (!e) return 1;
  const std::string s(e);
  return s == "off" ? 0 : s == "strict" ? 2 : 1;
}

PortChannel ProxyService::portChannel(SemaphoreId id, MemoryId dst, MemoryId src) {
  if (dst >= memories_.size() || src >= memories_.size())
    throw Error("ProxyService::portChannel: unknown memory id", ErrorCode::InvalidUsage);
  if (!memories_[dst].coherent()) {
    const int policy = portChannelDstPolicy();
    const std::string what = "PortChannel destination (memory id " + std::to_string(dst) + ", rank " +
                             std::to_string(memories_[dst].rank()) +
                             ") is cached device memory: what the proxy puts there is visible to the host and to "
                             "kernels launched after the receiving one, not to reads of a running kernel after "
                             "wait(); allocate it with GpuBuffer / mscclppAmdMallocUncached for that";
    if (policy == 2) throw Error(what + " (MSCCLPP_AMD_PORT_CHANNEL_DST=strict)", ErrorCode::InvalidUsage);
    if (policy == 1 && !warnedDst_) {
      warnedDst_ = true;
      host::warn(what);
    }
  }
  return PortChannel(id, semaphores_.at(id), proxy_, semConn_.at(id)->dFlushDone, dst, src);
}

void ProxyService::startProxy(bool blocking) { proxy_->start(blocking); }
void ProxyService::stopProxy() {
  if (proxy_) proxy_->stop();
}
int ProxyService::proxyNumaNode() const { return proxy_ ? proxy_->numaNode() : -1; }
uint64_t ProxyService::proxyMaxPollGapNs() const { return proxy_ ? proxy_->maxPollGapNs() : 0; }
void ProxyService::resetProxyPollGap() {
  if (proxy_) proxy_->resetPollGap();
}

namespace {
// A failure on the proxy thread becomes the device error word's code (first one wins on the host
// side; the kernel waiting on the missing data then sees a set word rather than only a timeout)
// and a warning with the reason.
void reportProxyFailure(uint32_t* err, const std::string& what) {
  host::warn("proxy: " + what);
  if (!err) return;
  // on a stream of its own: a kernel spinning for the data that never came must not delay it
  static hipStream_t s = [] {
    hipStream_t st = nullptr;
    (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    return st;
  }();
  (void)hipMemsetD32Async((hipDeviceptr_t)err, kErrProxyFailure, 1, s);
}
}  // namespace

static inline uint64_t steadyNs() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

ProxyHandlerResult ProxyService::handleTrigger(ProxyTrigger t, uint64_t pos) {
  ++handled_;
  const uint32_t id = (uint32_t)t.fields.semaphoreId;
  if (id >= semaphores_.size()) {
    reportProxyFailure(err_, "trigger names unknown semaphore " + std::to_string(id));
    return ProxyHandlerResult::Continue;
  }
  Host2DeviceSemaphore& sem = *semaphores_[id];
  Connection& conn = sem.connection();
  TriggerStamp* st = nullptr;
  if (stamps_.size() < stampCap_) {
    stamps_.emplace_back();
    st = &stamps_.back();
    st->type = (uint32_t)t.fields.type;
    st->seenNs = steadyNs();
  }
  try {
    if (t.fields.type & TriggerData) {
      const uint32_t d = (uint32_t)t.fields.dstMemoryId, s = (uint32_t)t.fields.srcMemoryId;
      if (d >= memories_.size() || s >= memories_.size())
        throw Error("trigger names an unknown memory id", ErrorCode::InvalidUsage);
      conn.write(memories_[d], t.fields.dstOffset, memories_[s], t.fields.srcOffset, t.fields.size);
      if (st) {
        st->dataNs = steadyNs();
        st->dataEvent = stampEvents_[2 * (stamps_.size() - 1)];
        (void)hipEventRecord((hipEvent_t)st->dataEvent, conn.stream());
      }
    }
    if (t.fields.type & TriggerFlag) {
      sem.signal();
      if (st) {
        st->flagNs = steadyNs();
        st->flagEvent = stampEvents_[2 * (stamps_.size() - 1) + 1];
        (void)hipEventRecord((hipEvent_t)st->flagEvent, conn.stream());
      }
    }
    if (t.fields.type & TriggerSync) {
      conn.flush();
      __atomic_store_n(semConn_[id]->flushDone, pos + 1, __ATOMIC_RELEASE);
    }
    if (st) st->doneNs = steadyNs();
  } catch (const std::exception& e) {
    reportProxyFailure(err_, e.what());
    if (t.fields.type & TriggerSync) __atomic_store_n(semConn_[id]->flushDone, pos + 1, __ATOMIC_RELEASE);
  }
  return ProxyHandlerResult::Continue;
}

BasePortChannel::DeviceHandle BasePortChannel::deviceHandle() const {
  const auto sh = semaphore_->deviceHandle();
  return DeviceHandle(semaphoreId_, sh, proxy_->fifo().deviceHandle(sh.budget, sh.err), flushDonePos_);
}

PortChannel::DeviceHandle PortChannel::deviceHandle() const {
  const auto sh = semaphore_->deviceHandle();
  return DeviceHandle(semaphoreId_, sh, proxy_->fifo().deviceHandle(sh.budget, sh.err), dst_, src_, flushDonePos_);
}

}  // namespace mscclpp_amd
