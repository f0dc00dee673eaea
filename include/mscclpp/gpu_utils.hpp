// <mscclpp/gpu_utils.hpp> on this library: gpuMemcpy / detail::gpuCallocShared / GpuBuffer.
// A caller written against the reference's include/mscclpp/gpu_utils.hpp compiles unchanged with
// `-I include`: the declarations live in mscclpp_amd/gpu_utils.hpp, and namespace mscclpp names them through
// a using-directive (qualified lookup of mscclpp::X finds mscclpp_amd::X; include/mscclpp/namespace.hpp).
#ifndef MSCCLPP_AMD_FWD_GPU_UTILS_HPP_
#define MSCCLPP_AMD_FWD_GPU_UTILS_HPP_

#include "mscclpp_amd/gpu_utils.hpp"
#include "mscclpp/namespace.hpp"

#endif  // MSCCLPP_AMD_FWD_GPU_UTILS_HPP_
