// <mscclpp/semaphore.hpp> on this library: Host2DeviceSemaphore / MemoryDevice2DeviceSemaphore.
// A caller written against the reference's include/mscclpp/semaphore.hpp compiles unchanged with
// `-I include`: the declarations live in mscclpp_amd/semaphore.hpp, and namespace mscclpp names them through
// a using-directive (qualified lookup of mscclpp::X finds mscclpp_amd::X; include/mscclpp/namespace.hpp).
#ifndef MSCCLPP_AMD_FWD_SEMAPHORE_HPP_
#define MSCCLPP_AMD_FWD_SEMAPHORE_HPP_

#include "mscclpp_amd/semaphore.hpp"
#include "mscclpp/namespace.hpp"

#endif  // MSCCLPP_AMD_FWD_SEMAPHORE_HPP_
