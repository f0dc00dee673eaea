// The proxy thread (include/mscclpp/proxy.hpp, src/core/proxy.cc:42-100): one host thread per
// Proxy, bound to the CPUs of the GPU's NUMA node (proxy.cc:23-33), busy-polling the FIFO and
// handing every trigger to a handler; the trigger is popped after the handler returns.
#ifndef MSCCLPP_AMD_PROXY_HPP_
#define MSCCLPP_AMD_PROXY_HPP_

#include <atomic>
#include <functional>
#include <memory>
#include <thread>

#include "mscclpp_amd/fifo.hpp"
#include "mscclpp_amd/numa.hpp"

namespace mscclpp_amd {

enum class ProxyHandlerResult { Continue, Stop };  // proxy.hpp:16-19

class Proxy {
 public:
  // handler(trigger, fifoPosition): the position is what the device's push() returned
  using Handler = std::function<ProxyHandlerResult(ProxyTrigger, uint64_t)>;
  Proxy(Handler handler, int fifoSize = DEFAULT_FIFO_SIZE);
  ~Proxy();
  Proxy(const Proxy&) = delete;
  Proxy& operator=(const Proxy&) = delete;
  void start(bool blocking = true);  // blocking: return once the thread runs
  void stop();
  Fifo& fifo() { return fifo_; }
  int numaNode() const { return numaNode_; }
  // The longest time (ns) the proxy thread went between two polls of the FIFO since the last reset:
  // a figure near the whole stall of an iteration means the thread was not running (host side).
  // Measured only with MSCCLPP_AMD_PROXY_GAP_STATS=1 (a clock read per poll), else 0.
  uint64_t maxPollGapNs() const { return maxGapNs_.load(std::memory_order_relaxed); }
  void resetPollGap() { resetGap_.store(true, std::memory_order_relaxed); }

 private:
  int device_ = 0;
  Fifo fifo_;
  Handler handler_;
  std::thread thread_;
  std::atomic<bool> running_{false};
  std::atomic<bool> started_{false};
  std::atomic<int> numaNode_{-1};
  std::atomic<uint64_t> maxGapNs_{0};
  std::atomic<bool> resetGap_{false};
};

}  // namespace mscclpp_amd

#endif  // MSCCLPP_AMD_PROXY_HPP_
