// <mscclpp/memory_channel.hpp> on this library: MemoryChannel (host side).
// A caller written against the reference's include/mscclpp/memory_channel.hpp compiles unchanged with
// `-I include`: the declarations live in mscclpp_amd/memory_channel.hpp, and namespace mscclpp names them through
// a using-directive (qualified lookup of mscclpp::X finds mscclpp_amd::X; include/mscclpp/namespace.hpp).
#ifndef MSCCLPP_AMD_FWD_MEMORY_CHANNEL_HPP_
#define MSCCLPP_AMD_FWD_MEMORY_CHANNEL_HPP_

#include "mscclpp_amd/memory_channel.hpp"
#include "mscclpp/namespace.hpp"

#endif  // MSCCLPP_AMD_FWD_MEMORY_CHANNEL_HPP_
