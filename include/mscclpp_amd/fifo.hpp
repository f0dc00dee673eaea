// Host side of the GPU -> host trigger FIFO (include/mscclpp/fifo.hpp:13-61, src/core/fifo.cc).
// The ring and the tail live in host-pinned, device-mapped coherent memory; head and the tail cache
// in device memory.  poll() accepts the slot at the tail only when its commit bit carries the
// parity of the tail's lap (fifo.cc:58-73), then clears the bit; pop() advances the tail with a
// release store (fifo.cc:75-78).  Single consumer (the proxy thread).
#ifndef MSCCLPP_AMD_FIFO_HPP_
#define MSCCLPP_AMD_FIFO_HPP_

#include <cstdint>

#include "mscclpp_amd/core.hpp"
#include "mscclpp_amd/fifo_device.hpp"

namespace mscclpp_amd {

constexpr int DEFAULT_FIFO_SIZE = 512;  // fifo.hpp:13

class Fifo {
 public:
  // size must be a power of two (Error with ErrorCode::InvalidUsage otherwise, fifo_tests.cu:155-162)
  explicit Fifo(int size = DEFAULT_FIFO_SIZE);
  ~Fifo();
  Fifo(const Fifo&) = delete;
  Fifo& operator=(const Fifo&) = delete;
  bool poll(ProxyTrigger& trigger);
  void pop();
  int size() const { return size_; }
  uint64_t tail() const;
  // budget / err: the wall-clock bound of the device's waits on a full ring and its error word
  FifoDeviceHandle deviceHandle(uint64_t budget = 0, uint32_t* err = nullptr) const;

 private:
  int size_;
  int shift_ = 0;
  ProxyTrigger* triggers_ = nullptr;
  ProxyTrigger* dTriggers_ = nullptr;
  uint64_t* tail_ = nullptr;
  uint64_t* dTail_ = nullptr;
  uint64_t* head_ = nullptr;
  uint64_t* tailCache_ = nullptr;
};

}  // namespace mscclpp_amd

#endif  // MSCCLPP_AMD_FIFO_HPP_
