// <mscclpp/semaphore_device.hpp> on this library: Host2DeviceSemaphoreDeviceHandle / MemoryDevice2DeviceSemaphoreDeviceHandle.
// A caller written against the reference's include/mscclpp/semaphore_device.hpp compiles unchanged with
// `-I include`: the declarations live in mscclpp_amd/semaphore_device.hpp, and namespace mscclpp names them through
// a using-directive (qualified lookup of mscclpp::X finds mscclpp_amd::X; include/mscclpp/namespace.hpp).
#ifndef MSCCLPP_AMD_FWD_SEMAPHORE_DEVICE_HPP_
#define MSCCLPP_AMD_FWD_SEMAPHORE_DEVICE_HPP_

#include "mscclpp_amd/semaphore_device.hpp"
#include "mscclpp/namespace.hpp"

#endif  // MSCCLPP_AMD_FWD_SEMAPHORE_DEVICE_HPP_
