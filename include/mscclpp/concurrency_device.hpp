// <mscclpp/concurrency_device.hpp> on this library: DeviceSyncer / DeviceSemaphore.
// A caller written against the reference's include/mscclpp/concurrency_device.hpp compiles unchanged with
// `-I include`: the declarations live in mscclpp_amd/concurrency_device.hpp, and namespace mscclpp names them through
// a using-directive (qualified lookup of mscclpp::X finds mscclpp_amd::X; include/mscclpp/namespace.hpp).
#ifndef MSCCLPP_AMD_FWD_CONCURRENCY_DEVICE_HPP_
#define MSCCLPP_AMD_FWD_CONCURRENCY_DEVICE_HPP_

#include "mscclpp_amd/concurrency_device.hpp"
#include "mscclpp/namespace.hpp"

#endif  // MSCCLPP_AMD_FWD_CONCURRENCY_DEVICE_HPP_
