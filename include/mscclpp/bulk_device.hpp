// <mscclpp/bulk_device.hpp> on this library (include/mscclpp_amd/bulk_device.hpp).
// A caller written against the reference's include/mscclpp/bulk_device.hpp compiles unchanged with
// `-I include`; namespace mscclpp names the declarations through a using-directive
// (include/mscclpp/namespace.hpp).
#ifndef MSCCLPP_AMD_FWD_BULK_DEVICE_HPP_
#define MSCCLPP_AMD_FWD_BULK_DEVICE_HPP_

#include "mscclpp_amd/bulk_device.hpp"
#include "mscclpp/namespace.hpp"

#endif  // MSCCLPP_AMD_FWD_BULK_DEVICE_HPP_
