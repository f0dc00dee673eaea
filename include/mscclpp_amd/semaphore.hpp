// Host-side semaphores (include/mscclpp/semaphore.hpp:16-115): the objects whose deviceHandle()
// kernels wait and signal on.
//   Host2DeviceSemaphore          signalled by this rank's host (the proxy), on behalf of the
//                                 connection's peer, with Connection::updateAndSync; waited on by
//                                 the peer's device (semaphore.cc:118-167)
//   MemoryDevice2DeviceSemaphore  signalled by a device thread with a system-scope atomic add into
//                                 the peer's token over xGMI (semaphore.cc:215-238)
// Device handles carry the communicator's spin budget and error word.  An error word passed
// explicitly (the `err` argument) must point at 4 words (16 bytes): a timed-out wait records the code
// in err[0] and its detail in err[1..3] (device.hpp report_error_detail).
#ifndef MSCCLPP_AMD_SEMAPHORE_HPP_
#define MSCCLPP_AMD_SEMAPHORE_HPP_

#include <memory>

#include "mscclpp_amd/core.hpp"
#include "mscclpp_amd/semaphore_device.hpp"

namespace mscclpp_amd {

class Host2DeviceSemaphore {
 public:
  Host2DeviceSemaphore(const Semaphore& semaphore, uint64_t budget = 0, uint32_t* err = nullptr);
  Host2DeviceSemaphore(Communicator& communicator, const Connection& connection);
  ~Host2DeviceSemaphore();
  Host2DeviceSemaphore(const Host2DeviceSemaphore&) = delete;
  Host2DeviceSemaphore& operator=(const Host2DeviceSemaphore&) = delete;
  Connection& connection();
  // Bump the outbound token and copy it into the peer's inbound token, ordered after every write
  // issued earlier on the connection.
  void signal();
  using DeviceHandle = Host2DeviceSemaphoreDeviceHandle;
  DeviceHandle deviceHandle() const;

 private:
  Semaphore semaphore_;
  uint64_t* expectedInboundToken_ = nullptr;  // device memory
  uint64_t* outboundSlots_ = nullptr;         // pinned host ring, one slot per signal value in flight
  uint64_t outbound_ = 0;
  uint64_t budget_ = 0;
  uint32_t* err_ = nullptr;
};

// Host2HostSemaphore (semaphore.hpp, semaphore.cc:169-214) pairs two CPU endpoints over a network
// transport; the reference refuses it on CudaIpc (:173-175), the only transport of one MI355X node,
// so here every constructor refuses it the same way (Error, InvalidUsage).
class Host2HostSemaphore {
 public:
  explicit Host2HostSemaphore(const Semaphore&) { refuse(); }
  Host2HostSemaphore(Communicator&, const Connection&) { refuse(); }
  Connection& connection() { refuse(); }
  void signal() { refuse(); }
  bool poll() { refuse(); }
  void wait(int64_t = 10000000) { refuse(); }

 private:
  [[noreturn]] static void refuse() {
    throw Error("Host2HostSemaphore cannot be used with CudaIpc transport", ErrorCode::InvalidUsage);
  }
};

class MemoryDevice2DeviceSemaphore {
 public:
  MemoryDevice2DeviceSemaphore(const Semaphore& semaphore, uint64_t budget = 0, uint32_t* err = nullptr);
  MemoryDevice2DeviceSemaphore(Communicator& communicator, const Connection& connection);
  ~MemoryDevice2DeviceSemaphore();
  MemoryDevice2DeviceSemaphore(const MemoryDevice2DeviceSemaphore&) = delete;
  MemoryDevice2DeviceSemaphore& operator=(const MemoryDevice2DeviceSemaphore&) = delete;
  Connection& connection();
  using DeviceHandle = MemoryDevice2DeviceSemaphoreDeviceHandle;
  DeviceHandle deviceHandle() const;

 private:
  Semaphore semaphore_;
  uint64_t* expectedInboundToken_ = nullptr;  // device memory
  uint64_t budget_ = 0;
  uint32_t* err_ = nullptr;
};

}  // namespace mscclpp_amd

#endif  // MSCCLPP_AMD_SEMAPHORE_HPP_
