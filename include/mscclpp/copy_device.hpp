// <mscclpp/copy_device.hpp> on this library: copy / copyToPackets / copyFromPackets.
// A caller written against the reference's include/mscclpp/copy_device.hpp compiles unchanged with
// `-I include`: the declarations live in mscclpp_amd/copy_device.hpp, and namespace mscclpp names them through
// a using-directive (qualified lookup of mscclpp::X finds mscclpp_amd::X; include/mscclpp/namespace.hpp).
#ifndef MSCCLPP_AMD_FWD_COPY_DEVICE_HPP_
#define MSCCLPP_AMD_FWD_COPY_DEVICE_HPP_

#include "mscclpp_amd/copy_device.hpp"
#include "mscclpp/namespace.hpp"

#endif  // MSCCLPP_AMD_FWD_COPY_DEVICE_HPP_
