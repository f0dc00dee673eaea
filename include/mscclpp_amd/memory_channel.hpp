// MemoryChannel host objects (include/mscclpp/memory_channel.hpp:16-82): a semaphore plus the
// destination (a peer's registered memory, mapped here), the source (local memory) and an optional
// local packet buffer the peer puts LL packets into.  deviceHandle() yields the
// MemoryChannelDeviceHandle of memory_channel_device.hpp.
#ifndef MSCCLPP_AMD_MEMORY_CHANNEL_HPP_
#define MSCCLPP_AMD_MEMORY_CHANNEL_HPP_

#include <memory>

#include "mscclpp_amd/core.hpp"
#include "mscclpp_amd/memory_channel_device.hpp"
#include "mscclpp_amd/semaphore.hpp"

namespace mscclpp_amd {

struct BaseMemoryChannel {
 protected:
  std::shared_ptr<MemoryDevice2DeviceSemaphore> semaphore_;

 public:
  BaseMemoryChannel() = default;
  BaseMemoryChannel(std::shared_ptr<MemoryDevice2DeviceSemaphore> semaphore) : semaphore_(std::move(semaphore)) {}
  BaseMemoryChannel(const Semaphore& semaphore);
  using DeviceHandle = BaseMemoryChannelDeviceHandle;
  DeviceHandle deviceHandle() const { return DeviceHandle(semaphore_->deviceHandle()); }
};

struct MemoryChannel : public BaseMemoryChannel {
 private:
  RegisteredMemory dst_;
  void* src_ = nullptr;
  RegisteredMemory srcMem_;
  void* packetBuffer_ = nullptr;

 public:
  MemoryChannel() = default;
  MemoryChannel(std::shared_ptr<MemoryDevice2DeviceSemaphore> semaphore, RegisteredMemory dst, RegisteredMemory src,
                void* packetBuffer = nullptr)
      : BaseMemoryChannel(std::move(semaphore)), dst_(dst), src_(src.data()), srcMem_(src), packetBuffer_(packetBuffer) {}
  MemoryChannel(const Semaphore& semaphore, RegisteredMemory dst, RegisteredMemory src, void* packetBuffer = nullptr)
      : BaseMemoryChannel(semaphore), dst_(dst), src_(src.data()), srcMem_(src), packetBuffer_(packetBuffer) {}
  // The earlier form with a plain local source pointer.
  MemoryChannel(std::shared_ptr<MemoryDevice2DeviceSemaphore> semaphore, RegisteredMemory dst, void* src,
                void* packetBuffer = nullptr)
      : BaseMemoryChannel(std::move(semaphore)), dst_(dst), src_(src), packetBuffer_(packetBuffer) {}
  using DeviceHandle = MemoryChannelDeviceHandle;
  DeviceHandle deviceHandle() const {
    return DeviceHandle(semaphore_->deviceHandle(), dst_.data(), src_, packetBuffer_);
  }
};

}  // namespace mscclpp_amd

#endif  // MSCCLPP_AMD_MEMORY_CHANNEL_HPP_
