// <mscclpp/core.hpp> on this library: Communicator / Connection / RegisteredMemory / Transport / Bootstrap.
// A caller written against the reference's include/mscclpp/core.hpp compiles unchanged with
// `-I include`: the declarations live in mscclpp_amd/core.hpp, and namespace mscclpp names them through
// a using-directive (qualified lookup of mscclpp::X finds mscclpp_amd::X; include/mscclpp/namespace.hpp).
#ifndef MSCCLPP_AMD_FWD_CORE_HPP_
#define MSCCLPP_AMD_FWD_CORE_HPP_

#include "mscclpp_amd/core.hpp"
#include "mscclpp/namespace.hpp"

#endif  // MSCCLPP_AMD_FWD_CORE_HPP_
