// PortChannels and the ProxyService behind them (include/mscclpp/port_channel.hpp:18-181,
// src/core/port_channel.cc).  Kernels push triggers naming a semaphore and two memory ids; the
// service's proxy thread turns them into Connection operations (port_channel.cc:117-178):
//   TriggerData  -> connection.write(memory[dst] + dstOffset, memory[src] + srcOffset, size)
//   TriggerFlag  -> the semaphore's signal() (updateAndSync of the peer's token)
//   TriggerSync  -> connection.flush(), then flushDonePos = position + 1 for the device's waitFlush
// A copy or token update that fails is reported through the communicator's device error word (so a
// kernel waiting on it learns of it through ncclCommGetAsyncError), not by a silent timeout.
#ifndef MSCCLPP_AMD_PORT_CHANNEL_HPP_
#define MSCCLPP_AMD_PORT_CHANNEL_HPP_

#include <memory>
#include <unordered_map>
#include <vector>

#include "mscclpp_amd/core.hpp"
#include "mscclpp_amd/port_channel_device.hpp"
#include "mscclpp_amd/proxy.hpp"
#include "mscclpp_amd/semaphore.hpp"

namespace mscclpp_amd {

struct BasePortChannel;
struct PortChannel;

class BaseProxyService {
 public:
  virtual ~BaseProxyService() = default;
  virtual void startProxy(bool blocking = false) = 0;
  virtual void stopProxy() = 0;
};

class ProxyService : public BaseProxyService {
 public:
  explicit ProxyService(int fifoSize = DEFAULT_FIFO_SIZE);
  ~ProxyService() override;
  SemaphoreId buildAndAddSemaphore(Communicator& communicator, const Connection& connection);
  SemaphoreId addSemaphore(const Semaphore& semaphore);
  SemaphoreId addSemaphore(std::shared_ptr<Host2DeviceSemaphore> semaphore);
  MemoryId addMemory(RegisteredMemory memory);
  MemoryId nextMemoryId(uint32_t count = 1) const;
  std::shared_ptr<Host2DeviceSemaphore> semaphore(SemaphoreId id) const;
  BasePortChannel basePortChannel(SemaphoreId id);
  PortChannel portChannel(SemaphoreId id, MemoryId dst, MemoryId src);
  void startProxy(bool blocking = false) override;
  void stopProxy() override;
  // Proxy thread's NUMA node (-1 before start or when unknown) and the number of triggers handled.
  int proxyNumaNode() const;
  uint64_t proxyMaxPollGapNs() const;  // Proxy::maxPollGapNs of this service's proxy thread
  void resetProxyPollGap();
  uint64_t triggersHandled() const { return handled_; }
  // Per-trigger stamps for latency analysis (off by default; the harnesses of DESIGN.md §9 turn them
  // on).  For each of the next `cap` triggers the proxy thread records the host clock when it got
  // the trigger and after it had submitted the data copy, the token update and the flush, plus HIP
  // events on the connection stream after the data copy and after the token update (the device
  // times at which they completed).  Call it with no trigger in flight (before startProxy, or once
  // the kernels pushing triggers have completed on every rank); read them after stopProxy(); the
  // events stay owned by the service until its destruction.
  struct TriggerStamp {
    uint32_t type = 0;       // TriggerData | TriggerFlag | TriggerSync bits of the trigger
    uint64_t seenNs = 0;     // steady clock when the handler started
    uint64_t dataNs = 0;     // after the data copy was submitted (0: no data)
    uint64_t flagNs = 0;     // after the token update was submitted (0: no flag)
    uint64_t doneNs = 0;     // handler end (after the flush for a sync trigger)
    void* dataEvent = nullptr;  // hipEvent_t recorded after the data copy (nullptr: none)
    void* flagEvent = nullptr;  // hipEvent_t recorded after the token update
  };
  void enableStamps(size_t cap);
  const std::vector<TriggerStamp>& stamps() const { return stamps_; }

 private:
  std::vector<TriggerStamp> stamps_;
  std::vector<void*> stampEvents_;  // hipEvent_t pool, 2 per stamp
  size_t stampCap_ = 0;
  struct ConnState;
  std::vector<std::shared_ptr<Host2DeviceSemaphore>> semaphores_;
  std::vector<RegisteredMemory> memories_;
  bool warnedDst_ = false;  // a non-coherent PortChannel destination was reported (channels.cpp)
  std::unordered_map<const void*, std::shared_ptr<ConnState>> conns_;  // per connection: flushDonePos
  std::vector<std::shared_ptr<ConnState>> semConn_;                    // per semaphore id
  std::shared_ptr<Proxy> proxy_;
  uint32_t* err_ = nullptr;  // device error word of the communicator the semaphores came from
  uint64_t budget_ = 0;
  uint64_t handled_ = 0;
  ProxyHandlerResult handleTrigger(ProxyTrigger trigger, uint64_t pos);
  friend struct BasePortChannel;
  friend struct PortChannel;
};

struct BasePortChannel {
 protected:
  SemaphoreId semaphoreId_ = 0;
  std::shared_ptr<Host2DeviceSemaphore> semaphore_;
  std::shared_ptr<Proxy> proxy_;
  uint64_t* flushDonePos_ = nullptr;  // device pointer of the connection's pinned flush position

 public:
  BasePortChannel() = default;
  BasePortChannel(SemaphoreId semaphoreId, std::shared_ptr<Host2DeviceSemaphore> semaphore, std::shared_ptr<Proxy> proxy,
                  uint64_t* flushDonePos)
      : semaphoreId_(semaphoreId), semaphore_(std::move(semaphore)), proxy_(std::move(proxy)),
        flushDonePos_(flushDonePos) {}
  using DeviceHandle = BasePortChannelDeviceHandle;
  DeviceHandle deviceHandle() const;
};

struct PortChannel : public BasePortChannel {
 private:
  MemoryId dst_ = 0;
  MemoryId src_ = 0;

 public:
  PortChannel() = default;
  PortChannel(SemaphoreId semaphoreId, std::shared_ptr<Host2DeviceSemaphore> semaphore, std::shared_ptr<Proxy> proxy,
              uint64_t* flushDonePos, MemoryId dst, MemoryId src)
      : BasePortChannel(semaphoreId, std::move(semaphore), std::move(proxy), flushDonePos), dst_(dst), src_(src) {}
  using DeviceHandle = PortChannelDeviceHandle;
  DeviceHandle deviceHandle() const;
};

}  // namespace mscclpp_amd

#endif  // MSCCLPP_AMD_PORT_CHANNEL_HPP_
